"""Typed configuration slots: ``Field`` and ``ComponentField``.

Behavioural parity with zookeeper/core/field.py (``Field`` :13-172,
``ComponentField`` :178-281): same constructor contract, same error texts,
same ``__set_name__`` annotation lookup along the MRO and the same
``has_default`` / ``get_default`` semantics.

Design difference (MI355X-first, hot-path aware): the reference resolves a
field through a wrapped ``__getattribute__`` on every attribute access
(≈1.3 µs per cached read, zookeeper/core/component.py:148-198).  Here a field
is a *non-data descriptor*: the first read on an instance calls ``__get__``,
which resolves the value (configured → ``__init__`` kwarg → default →
inherited), type-checks it and stores it in the instance ``__dict__``.  Every
later read is an ordinary instance-dict hit with no Python-level code at all,
so component fields can be read inside a training loop at plain-attribute cost.
"""

from __future__ import annotations

import inspect
from typing import Any, Callable, Generic, Optional, Type, TypeVar, Union

from zookeeper_amd.core import utils
from zookeeper_amd.core.partial_component import PartialComponent

C = TypeVar("C")  # host component type
F = TypeVar("F")  # field value type

# Installed by `zookeeper_amd.core.component` at import time; resolves a field
# value for an instance (see `component._public_value`).
_instance_resolver: Optional[Callable[[Any, str], Any]] = None

_FIELD_DEFAULT_ERROR = (
    "If `default` is passed to `Field`, it must be either:\n"
    "- An immutable value (int, float, bool, string, or None).\n"
    "- A function or lambda accepting no arguments or a single\n"
    "  argument (`self`), and returning the default value.\n"
    "Received: {default}."
)

_FIELD_ANNOTATION_ERROR = (
    "Fields must be defined inside the component class definition, "
    "with a type annotation in one of the following ways:\n\n"
    "```\n"
    "@component\n"
    "class ComponentClass:\n"
    "    ...\n"
    "    # Like this\n"
    "    name_1: type_1 = Field(default_1)\n"
    "    ...\n"
    "    # Or like this\n"
    "    @Field\n"
    "    def name_2(self) -> type_2:\n"
    "        ...\n"
    "        return default_2\n"
    "```\n\n"
    "Unable to find a type annotation for field '{name}' on class '{cls}'."
)

_COMPONENT_FIELD_ANNOTATION_ERROR = (
    "ComponentFields must be defined inside the component class definition, "
    "with a type-annotation as follows:\n\n"
    "```\n"
    "@component\n"
    "class ParentComponentClass:\n"
    "    field_name: SomeChildComponentType = ComponentField(\n"
    "        SomeDefaultChildComponentClass\n"
    "    )\n"
    "```\n"
    "\nUnlike `Field`, `ComponentField` cannot be used as a decorator.\n\n"
    "Unable to find a type annotation for field '{name}' on class '{cls}'."
)


def _annotation_along_mro(cls: type, name: str) -> Any:
    for klass in inspect.getmro(cls):
        annotations = vars(klass).get("__annotations__", {})
        if name in annotations:
            return annotations[name]
    return utils.missing


def _accepts_at_most_self(fn: Callable) -> bool:
    params = list(inspect.signature(fn).parameters.values())
    if len(params) > 1:
        return False
    if len(params) == 1 and params[0].kind in (
        inspect.Parameter.VAR_POSITIONAL,
        inspect.Parameter.VAR_KEYWORD,
    ):
        return False
    return True


class Field(Generic[C, F]):
    """A typed, configurable slot on a component.

    ``default`` may be ``missing`` (no default), an immutable value, or a
    function of zero arguments or of ``self``.  ``Field`` can also decorate a
    method, whose return annotation becomes the field type::

        @Field
        def optimizer(self) -> Optimizer:
            return Adam(self.learning_rate)
    """

    def __init__(
        self,
        default: Union[utils.Missing, F, Callable[[], F], Callable[[C], F]] = utils.missing,
        *,
        allow_missing: bool = False,
    ):
        self.name: Any = None
        self.type: Any = None
        self.host_component_class: Any = None
        self.allow_missing = allow_missing
        self._registered = False
        self._return_annotation: Any = inspect.Signature.empty

        if allow_missing and default is not utils.missing:
            raise ValueError(
                "If a `Field` has `allow_missing=True`, no default can be provided."
            )
        if default is utils.missing or utils.is_immutable(default):
            self._default = default
            return
        if inspect.isfunction(default) and _accepts_at_most_self(default):
            self._default = default
            self._return_annotation = inspect.signature(default).return_annotation
            return
        raise TypeError(_FIELD_DEFAULT_ERROR.format(default=default))

    # -- PEP 487 ----------------------------------------------------------- #

    def _check_registrable(self, name: str) -> None:
        if self._registered:
            raise ValueError("This field has already been registered to a component.")
        if name.startswith("_"):
            raise ValueError("Field names cannot start with underscores.")

    def _register(self, host: type, name: str, annotation: Any) -> None:
        self.name = name
        self.host_component_class = host
        self.type = annotation
        self._registered = True

    def __set_name__(self, host: Type[C], name: str) -> None:
        self._check_registrable(name)
        annotation = _annotation_along_mro(host, name)
        ret = self._return_annotation
        if ret is not inspect.Signature.empty:
            if annotation is not utils.missing and annotation != ret:
                raise TypeError(
                    f"Two non-equal type annotations found for field '{name}': "
                    f"{annotation} and {ret}."
                )
            annotation = ret
        if annotation is utils.missing:
            raise TypeError(_FIELD_ANNOTATION_ERROR.format(name=name, cls=host.__name__))
        self._register(host, name, annotation)

    # -- descriptor protocol (non-data: instance __dict__ wins once cached) -- #

    def __get__(self, instance: Any, owner: Optional[type] = None) -> Any:
        if instance is None:
            return self
        fields = getattr(type(instance), "__component_fields__", None)
        if fields is None or self.name not in fields or _instance_resolver is None:
            # A Field on a plain (non-component) class behaves like an ordinary
            # class attribute, exactly as in the reference.
            return self
        return _instance_resolver(instance, self.name)

    # -- introspection ----------------------------------------------------- #

    def __repr__(self) -> str:
        if not self._registered:
            return "<Unregistered Field>"
        return (
            f"<Field '{self.name}' of {self.host_component_class.__name__} with type "
            f"{self.type}>"
        )

    def _require_registered(self) -> None:
        if not self._registered:
            raise ValueError("This field has not been registered to a component.")

    @property
    def has_default(self) -> bool:
        self._require_registered()
        return self._default is not utils.missing

    def _check_host(self, instance: Any, label: str) -> None:
        host = self.host_component_class
        if not isinstance(instance, host):
            raise TypeError(
                f"{label} '{self.name}' belongs to component '{host.__name__}'; "
                f"`get_default` must be called with an instance of '{host.__name__}'. "
                f"Received: {repr(instance)}."
            )

    def get_default(self, instance: C) -> F:
        self._require_registered()
        if not self.has_default:
            raise AttributeError(f"Field '{self.name}' has no default or configured value.")
        self._check_host(instance, "Field")

        default = self._default
        if not inspect.isfunction(default):
            return default
        if inspect.signature(default).parameters:
            value = default(instance)
        else:
            value = default()
        if utils.is_component_instance(value):
            raise TypeError(
                f"Field '{self.name}' of component '{instance.__component_name__}' "
                "is returning a component instance as its default value. To use "
                "components in fields, use `ComponentField` rather than `Field`."
            )
        return value


class ComponentField(Field, Generic[C, F]):
    """A slot holding a nested sub-component.

    ``default`` is a component (or @factory) class or a ``PartialComponent``;
    extra keyword arguments turn a class default into a ``PartialComponent``.
    The default is instantiated fresh (and unconfigured) for every host
    instance; the child then inherits missing values from its parents.
    """

    def __init__(
        self,
        default: Union[utils.Missing, F, PartialComponent] = utils.missing,
        *,
        allow_missing: bool = False,
        **kwargs: Any,
    ):
        if allow_missing and default is not utils.missing:
            raise ValueError(
                "If a `Field` has `allow_missing=True`, no default can be provided."
            )
        if default is utils.missing:
            if kwargs:
                raise TypeError(
                    "Keyword arguments can only be passed to `ComponentField` if "
                    "a default component class is also passed."
                )
        elif isinstance(default, PartialComponent) or utils.is_component_class(default):
            if kwargs:
                default = PartialComponent(default, **kwargs)
        elif utils.is_component_instance(default):
            raise TypeError(
                "The `default` passed to `ComponentField` must be a component class, "
                f"not a component instance. Received: {repr(default)}."
            )
        else:
            raise TypeError(
                "The `default` passed to `ComponentField` must be either a component "
                "class or a `PartialComponent`."
            )

        self.name = utils.missing
        self.type = utils.missing
        self.host_component_class = utils.missing
        self.allow_missing = allow_missing
        self._registered = False
        self._return_annotation = inspect.Signature.empty
        self._default = default

    def __set_name__(self, host: Type[C], name: str) -> None:
        self._check_registrable(name)
        annotation = _annotation_along_mro(host, name)
        if annotation is utils.missing:
            raise TypeError(
                _COMPONENT_FIELD_ANNOTATION_ERROR.format(name=name, cls=host.__name__)
            )
        self._register(host, name, annotation)

    def get_default(self, instance: C) -> F:
        self._require_registered()
        if not self.has_default:
            raise AttributeError(
                f"ComponentField '{self.name}' has no default or configured component "
                "class."
            )
        self._check_host(instance, "ComponentField")
        # A fresh, unconfigured child; it picks up missing values from its
        # parents once it is attached during `configure`.
        return self._default()
