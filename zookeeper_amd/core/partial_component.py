"""``PartialComponent``: ``functools.partial`` for component classes.

Parity: zookeeper/core/partial_component.py:26-116 (argument validation, lazy
kwargs, the class-body guard and call-time overrides).
"""

from __future__ import annotations

import inspect
from typing import Any, Callable, Dict, Generic, Type, TypeVar

from zookeeper_amd.core import utils

_T = TypeVar("_T")

_KWARGS_ERROR = (
    "Keyword arguments passed to `PartialComponent` must be either:\n"
    "- An immutable value (int, float, bool, string, or None).\n"
    "- A function or lambda accepting no arguments and returning the value that "
    "should be passed to the component upon instantiation.\n"
    "- An @component class that will be used to instantiate a component instance "
    "for the corresponding field value.\n"
    "- Another `PartialComponent`.\n"
    "Wrapping non-immutable values in a function / lambda allows the values "
    "to be lazily evaluated; they won't be created at all if the partial "
    "component is never instantiated."
)

_CLASS_BODY_ERROR = (
    "`PartialComponent` instances should not be directly assigned to class "
    "bodies. You should instead use `PartialComponent` inside a "
    "`ComponentField`, like so:\n"
    "```\n"
    "@component\n"
    "class ParentComponentClass:\n"
    "    child_component: SomeChildComponentType = ComponentField(\n"
    "        PartialComponent(\n"
    "            SomeDefaultChildComponentClass,\n"
    "            some_arg=some_default_value,\n"
    "            some_other_arg=some_other_default_value,\n"
    "            ...\n"
    "        )\n"
    "    )\n"
    "```"
)


def _unknown_kwarg(name: str, cls: type) -> TypeError:
    return TypeError(
        f"Keyword argument '{name}' passed to `PartialComponent` does not correspond "
        f"to any field of component class '{cls.__name__}'."
    )


def _as_thunk(value: Any) -> Callable[[], Any]:
    """Turn an accepted kwarg value into a zero-argument callable (or keep a
    component class / nested partial, both of which are already callable)."""
    if utils.is_immutable(value):
        return utils.wrap_in_callable(value)
    if utils.is_component_class(value) or isinstance(value, PartialComponent):
        return value
    if inspect.isfunction(value) and not inspect.signature(value).parameters:
        return value
    raise TypeError(_KWARGS_ERROR)


class PartialComponent(Generic[_T]):
    """``PartialComponent(Cls, a=3)(b=4)`` is equivalent to ``Cls(a=3, b=4)``."""

    def __init__(self, component_class: Type[_T], **kwargs: Any):
        if utils.is_component_instance(component_class):
            raise TypeError(
                "`PartialComponent` must be passed component classes, not component "
                f"instances. Received: {repr(component_class)}"
            )
        if not utils.is_component_class(component_class):
            raise TypeError(
                "The class passed to `PartialComponent` must be a component class. "
                f"Received: {component_class}."
            )
        if not kwargs:
            raise TypeError("`PartialComponent` must receive at least one keyword argument.")

        fields = component_class.__component_fields__
        thunks: Dict[str, Callable[[], Any]] = {}
        for name, value in kwargs.items():
            if name not in fields:
                raise _unknown_kwarg(name, component_class)
            thunks[name] = _as_thunk(value)

        self._component_class = component_class
        self._lazy_kwargs = thunks

    def __set_name__(self, owner: type, name: str) -> None:
        raise ValueError(_CLASS_BODY_ERROR)

    @property
    def component_class(self) -> type:
        return self._component_class

    def __call__(self, **overrides: Any) -> _T:
        cls = self._component_class
        for name in overrides:
            if name not in cls.__component_fields__:
                raise _unknown_kwarg(name, cls)
        # Only evaluate the saved thunks that are not overridden.
        merged = {n: t() for n, t in self._lazy_kwargs.items() if n not in overrides}
        merged.update(overrides)
        return cls(**merged)

    def __repr__(self) -> str:
        args = ", ".join(self._lazy_kwargs)
        return f"PartialComponent({self._component_class.__name__}, {args})"
