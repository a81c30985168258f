"""The ``@factory`` decorator.

A factory is a component with an argument-less ``build(self) -> T`` method.
When a factory instance is the value of a field, reading that field returns
``build()``'s result (built once, lazily, and type-checked against ``T``),
while configuration code still sees the factory itself via ``base_getattr``.

Parity: zookeeper/core/factory.py:10-131 (validation, error texts, the
run-once ``build`` wrapper, "Unconfigured factory" strings and registration
under the return annotation).
"""

from __future__ import annotations

import functools
import inspect
from typing import Any, Type

from zookeeper_amd.core import utils
from zookeeper_amd.core.component import component
from zookeeper_amd.core.factory_registry import FACTORY_REGISTRY, register_factory

__all__ = ["factory", "FACTORY_REGISTRY"]

_BUILD_SIGNATURE_ERROR = (
    "Classes decorated with @factory must implement a `build()` method taking "
    "precisely one positional argument, `self`."
)

_BUILD_RETURN_ERROR = (
    "The `build()` method of a @factory class must have an annotated return "
    "type annotation, e.g.:\n\n"
    "```\n"
    "@factory\n"
    "class MyFactory:\n"
    "    ...\n"
    "    def build(self) -> SomeReturnType:\n"
    "        ...\n"
    "        return some_value\n"
    "```"
)

_VALUE_ATTR = "__component_factory_value__"


def _build_signature(cls: type) -> inspect.Signature:
    build = getattr(cls, "build", None)
    if build is None:
        raise TypeError(_BUILD_SIGNATURE_ERROR)
    try:
        sig = inspect.signature(build)
    except (TypeError, ValueError):
        raise TypeError(_BUILD_SIGNATURE_ERROR) from None
    params = list(sig.parameters.values())
    if (
        len(params) != 1
        or params[0].name != "self"
        or params[0].kind in (inspect.Parameter.VAR_POSITIONAL, inspect.Parameter.VAR_KEYWORD)
    ):
        raise TypeError(_BUILD_SIGNATURE_ERROR)
    return sig


def _memoised_build(cls: type, build: Any):
    @functools.wraps(build)
    def build_once(self):
        cached = self.__dict__.get(_VALUE_ATTR, utils.missing)
        if cached is utils.missing:
            result = build(self)
            ret = cls.__component_factory_return_type__
            if not utils.type_check(result, ret):
                raise TypeError(
                    f"@factory '{cls}' has a `build()` method annotated with return "
                    f"type {ret}, which is not satisfied by the return value {result}."
                )
            self.__dict__[_VALUE_ATTR] = cached = result
        return cached

    return build_once


def _relabel(fn: Any):
    @functools.wraps(fn)
    def relabelled(self):
        return fn(self).replace("<Unconfigured component ", "<Unconfigured factory ")

    return relabelled


def factory(cls: Type) -> Type:
    """Turn a class with ``build(self) -> T`` into a factory component."""
    cls = component(cls)
    sig = _build_signature(cls)
    if sig.return_annotation is inspect.Signature.empty:
        raise TypeError(_BUILD_RETURN_ERROR)

    ret = sig.return_annotation
    if isinstance(ret, str):
        # PEP 563 string annotation: resolve in the defining module.
        try:
            ret = eval(ret, getattr(cls.build, "__globals__", {}), dict(vars(cls)))  # noqa: S307
        except Exception:
            pass
    cls.__component_factory_return_type__ = ret
    cls.__component_factory_value__ = utils.missing
    cls.build = _memoised_build(cls, cls.build)
    cls.__str__ = _relabel(cls.__str__)
    cls.__repr__ = _relabel(cls.__repr__)
    register_factory(ret, cls)
    return cls
