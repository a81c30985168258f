"""The ``@component`` decorator and ``configure``.

Components are classes with typed ``Field``s (plain values) and
``ComponentField``s (nested sub-components).  After instantiation a tree of
components is *configured* from a flat dict of dotted keys; values are
injected top-down with **scoped inheritance**: a child that declares a field
with the same name as an ancestor receives the ancestor's value unless a value
is configured on the child itself or on a closer ancestor::

    @component
    class A:
        x: int = Field()

    @component
    class B:
        a: A = ComponentField(A)
        x: int = Field()

    b = B()
    configure(b, {"x": 5, "a.x": 7})   # b.x == 5, b.a.x == 7
    configure(B2 := B(), {"x": 5})     # B2.a.x == 5 (inherited)

Behavioural parity (reference file:line):

* value precedence (configured on self/nearest ancestor > ``__init__`` kwarg >
  own default > nearest ancestor's value) .... zookeeper/core/component.py:115-198
* implicit ``build()`` of @factory values ....... zookeeper/core/component.py:215-222
* set/delete guards, ``dir`` .................... zookeeper/core/component.py:235-277
* ``str``/``repr`` formats ...................... zookeeper/core/component.py:286-337
* ``__init__`` contract ......................... zookeeper/core/component.py:345-372
* decorator validation .......................... zookeeper/core/component.py:380-458
* ``configure`` algorithm and error texts ....... zookeeper/core/component.py:461-695

Implementation notes (differences that are not behavioural):

* Field values are resolved by the ``Field`` descriptor on first access and
  then live in the instance ``__dict__`` (see ``field.py``): a cached read is a
  plain attribute read.  The *raw* resolved value (the @factory instance rather
  than its ``build()`` product) is kept in ``__component_raw_values__`` for
  ``base_getattr``.
* ``configure`` does not consume keys from the caller's dict (the reference
  mutates it as a side effect).
* Assigning a field before configuration invalidates a previously cached read.
"""

from __future__ import annotations

import inspect
from typing import Any, Dict, Iterator, List, Optional, Type

from zookeeper_amd.core import field as _field_module
from zookeeper_amd.core import utils
from zookeeper_amd.core.factory_registry import FACTORY_REGISTRY
from zookeeper_amd.core.field import ComponentField, Field

INDENT = " " * 4

# Per-instance bookkeeping attribute names (dunder names, never fields).
_INIT_VALUES = "__component_instantiated_field_values__"
_CONF_VALUES = "__component_configured_field_values__"
_IN_SCOPE = "__component_fields_with_values_in_scope__"
_RAW_VALUES = "__component_raw_values__"

_KEY_ERROR_HINT = (
    "\n\n"
    "If you have nested components as follows:\n\n"
    "```\n"
    "@component\n"
    "class ChildComponent:\n"
    "    a: int = Field(0)\n"
    "\n"
    "@task\n"
    "class SomeTask:\n"
    "    child: ChildComponent = ComponentField(ChildComponent)\n"
    "    def run(self):\n"
    "        print(self.child.a)\n"
    "```\n\n"
    "then trying to configure `a=<SOME_VALUE>` will fail. You instead need to "
    "fully qualify the key name, and configure the value with "
    "`child.a=<SOME_VALUE>`."
)


# --------------------------------------------------------------------------- #
# Value resolution
# --------------------------------------------------------------------------- #


def _checked(instance: Any, field: Field, value: Any) -> Any:
    if not utils.type_check(value, field.type):
        raise TypeError(
            f"Field '{field.name}' of component '{instance.__component_name__}' is "
            f"annotated with type '{field.type}', which is not satisfied by "
            f"value {repr(value)}."
        )
    return value


def _raw_value(instance: Any, name: str) -> Any:
    """Resolve (and cache) the raw value of field ``name`` without calling
    ``build()`` on @factory values.  Raises ``AttributeError`` if there is no
    value anywhere in scope."""
    d = instance.__dict__
    raw_cache = d.get(_RAW_VALUES)
    if raw_cache is not None and name in raw_cache:
        return raw_cache[name]

    fields = type(instance).__component_fields__
    field = fields[name]

    # 1) A configured value on this instance or the nearest declaring ancestor.
    for node in utils.generate_component_ancestors_with_field(
        instance, name, include_instance=True
    ):
        conf = node.__dict__.get(_CONF_VALUES)
        if conf is not None and name in conf:
            value = _checked(instance, field, conf[name])
            d.get(_INIT_VALUES, {}).pop(name, None)
            return _remember(instance, name, value)

    # 2) A value passed to this instance's `__init__` (or set before configure).
    init_values = d.get(_INIT_VALUES)
    if init_values is not None and name in init_values:
        return _remember(instance, name, _checked(instance, field, init_values[name]))

    # 3) The field default, else the nearest declaring ancestor's value.
    try:
        value = field.get_default(instance)
    except AttributeError as no_default:
        parent = next(utils.generate_component_ancestors_with_field(instance, name), None)
        if parent is None:
            raise no_default from None
        try:
            value = _raw_value(parent, name)
        except AttributeError:
            raise no_default from None
    return _remember(instance, name, _checked(instance, field, value))


def _remember(instance: Any, name: str, value: Any) -> Any:
    d = instance.__dict__
    raw_cache = d.get(_RAW_VALUES)
    if raw_cache is None:
        raw_cache = d[_RAW_VALUES] = {}
    raw_cache[name] = value
    if not utils.is_factory_instance(value):
        # Non-factory values are also the public value: cache them in the
        # instance dict so that later reads bypass the descriptor entirely.
        d[name] = value
    return value


def _public_value(instance: Any, name: str) -> Any:
    """Descriptor entry point (``instance.name``): the raw value, with
    @factory values replaced by their (cached) ``build()`` result."""
    value = _raw_value(instance, name)
    if utils.is_factory_instance(value):
        value = value.build()
        instance.__dict__[name] = value
    return value


_field_module._instance_resolver = _public_value


def base_getattr(instance: Any, name: str) -> Any:
    """Like ``getattr`` but returns @factory instances un-built (parity:
    zookeeper/core/component.py:229-232)."""
    if utils.is_component_instance(instance) and name in type(instance).__component_fields__:
        return _raw_value(instance, name)
    return getattr(instance, name)


def _invalidate(instance: Any, name: str) -> None:
    instance.__dict__.pop(name, None)
    raw = instance.__dict__.get(_RAW_VALUES)
    if raw is not None:
        raw.pop(name, None)


# --------------------------------------------------------------------------- #
# Methods installed on component classes
# --------------------------------------------------------------------------- #


def _component_init(self, **kwargs: Any) -> None:
    fields = type(self).__component_fields__
    for name in kwargs:
        if name not in fields:
            raise TypeError(
                "Keyword arguments passed to component `__init__` must correspond to "
                f"component fields. Received non-matching argument '{name}'."
            )
    d = self.__dict__
    d[_INIT_VALUES] = dict(kwargs)
    d[_CONF_VALUES] = {}
    d[_IN_SCOPE] = {n for n, f in fields.items() if f.has_default} | set(kwargs)


def _component_setattr(self, name: str, value: Any) -> None:
    if name in type(self).__component_fields__:
        if self.__component_configured__:
            raise ValueError(
                "Setting already configured component field values directly is "
                "prohibited. Use Zookeeper component configuration to set field"
                " values."
            )
        self.__dict__[_INIT_VALUES][name] = value
        _invalidate(self, name)
        return
    object.__setattr__(self, name, value)


def _component_delattr(self, name: str) -> None:
    if name in type(self).__component_fields__:
        raise ValueError("Deleting component field values is prohibited.")
    object.__delattr__(self, name)


def _component_dir(self) -> List[str]:
    return sorted(set(object.__dir__(self)) | set(type(self).__component_fields__))


def _field_strings(instance: Any, single_line: bool) -> Iterator[str]:
    for name, field in type(instance).__component_fields__.items():
        try:
            value = base_getattr(instance, name)
        except AttributeError:
            if not field.allow_missing:
                raise
            value = utils.missing

        inherited = False
        parent = next(utils.generate_component_ancestors_with_field(instance, name), None)
        if value is not utils.missing and parent is not None:
            try:
                inherited = base_getattr(parent, name) is value
            except AttributeError:
                inherited = False

        if utils.is_component_instance(value):
            if inherited:
                text = "<inherited component instance>"
            elif single_line:
                text = repr(value)
            else:
                text = f"\n{INDENT}".join(str(value).split("\n"))
        elif inherited:
            text = "<inherited value>"
        elif callable(value):
            text = "<callable>"
        elif isinstance(value, str):
            text = f'"{value}"'
        else:
            text = f"{value}"
        yield f"{name}={text}"


def flatten_config(instance: Any, prefix: str = "") -> Dict[str, Any]:
    """The resolved configuration of a configured component tree as a flat
    dotted-key dict — the same key syntax ``configure`` and the CLI accept,
    so a run record (``config.json``) can be replayed.  A sub-component
    contributes ``key: ClassName`` plus its own fields under ``key.``; values
    a child inherits from an ancestor are recorded once, at the ancestor;
    missing ``allow_missing`` fields are omitted; callables are recorded by
    name.  Not in the reference (its only record is ``str(task)``,
    zookeeper/core/component.py:331-337)."""
    out: Dict[str, Any] = {}
    for name, field in type(instance).__component_fields__.items():
        try:
            value = base_getattr(instance, name)
        except AttributeError:
            continue
        parent = next(utils.generate_component_ancestors_with_field(instance, name), None)
        if parent is not None:
            try:
                if base_getattr(parent, name) is value:
                    continue
            except AttributeError:
                pass
        key = prefix + name
        if utils.is_component_instance(value):
            out[key] = type(value).__name__
            out.update(flatten_config(value, key + "."))
        elif callable(value) and not isinstance(value, type):
            out[key] = f"<callable {getattr(value, '__qualname__', type(value).__name__)}>"
        elif isinstance(value, type):
            out[key] = value.__name__
        else:
            out[key] = value
    return out


def _unconfigured(instance: Any) -> str:
    return f"<Unconfigured component '{instance.__component_name__}' instance>"


def _component_repr(self) -> str:
    if not self.__component_configured__:
        return _unconfigured(self)
    return f"{type(self).__name__}({', '.join(_field_strings(self, True))})"


def _component_str(self) -> str:
    if not self.__component_configured__:
        return _unconfigured(self)
    body = f",\n{INDENT}".join(_field_strings(self, False))
    return f"{type(self).__name__}(\n{INDENT}{body}\n)"


# --------------------------------------------------------------------------- #
# The decorator
# --------------------------------------------------------------------------- #


def _validate_post_configure(cls: type) -> None:
    if not hasattr(cls, "__post_configure__"):
        return
    hook = cls.__post_configure__
    if not callable(hook):
        raise TypeError(
            "The `__post_configure__` attribute of a @component class must be a method."
        )
    params = inspect.signature(hook).parameters
    if len(params) > 1 or (len(params) == 1 and "self" not in params):
        raise TypeError(
            "The `__post_configure__` method of a @component class must take no "
            f"arguments except `self`, but `{cls.__name__}.__post_configure__` "
            f"accepts arguments {tuple(params)}."
        )


def _collect_fields(cls: type) -> Dict[str, Field]:
    fields: Dict[str, Field] = {}
    for klass in reversed(inspect.getmro(cls)):
        for name, value in vars(klass).items():
            if isinstance(value, Field):
                fields[name] = value
    return fields


def _resolve_string_annotations(cls: type, fields: Dict[str, Field]) -> None:
    """Resolve PEP 563 (``from __future__ import annotations``) string
    annotations against the defining module, when possible.  Unresolvable
    names (e.g. classes local to a function) stay strings and are then not
    type-checked."""
    import sys

    module_ns = vars(sys.modules.get(cls.__module__, object())) if cls.__module__ else {}
    for f in fields.values():
        if isinstance(f.type, str):
            try:
                f.type = eval(f.type, dict(module_ns), dict(vars(cls)))  # noqa: S307
            except Exception:
                pass


def component(cls: Type) -> Type:
    """Turn a class into a component (see the module docstring)."""
    if not inspect.isclass(cls):
        raise TypeError("Only classes can be decorated with @component.")
    if inspect.isabstract(cls):
        raise TypeError("Abstract classes cannot be decorated with @component.")
    if utils.is_component_class(cls):
        raise TypeError(
            f"The class {cls.__name__} is already a component; the @component decorator "
            "cannot be applied again."
        )
    if cls.__init__ not in (object.__init__, _component_init):
        raise TypeError("Component classes must not define a custom `__init__` method.")
    _validate_post_configure(cls)

    fields = _collect_fields(cls)
    _resolve_string_annotations(cls, fields)
    if not fields:
        utils.warn(f"Component {cls.__name__} has no defined fields.")

    for name in dir(cls):
        if name in fields and not isinstance(getattr(cls, name), Field):
            sup = fields[name].host_component_class
            raise ValueError(
                f"Field '{name}' is defined on super-class {sup.__name__}. "
                f"In subclass {cls.__name__}, '{name}' has been overriden with value: "
                f"{getattr(cls, name)}.\n\n"
                f"If you wish to change the default value of field '{name}' in a "
                f"subclass of {sup.__name__}, please wrap the new default "
                "value in a new `Field` instance."
            )

    cls.__init__ = _component_init
    cls.__setattr__ = _component_setattr
    cls.__delattr__ = _component_delattr
    cls.__dir__ = _component_dir
    cls.__str__ = _component_str
    cls.__repr__ = _component_repr
    cls.__component_fields__ = fields
    cls.__component_name__ = cls.__name__
    cls.__component_parent__ = None
    cls.__component_configured__ = False
    return cls


# --------------------------------------------------------------------------- #
# configure
# --------------------------------------------------------------------------- #


def _type_label(tp: Any) -> str:
    return tp.__name__ if inspect.isclass(tp) else str(tp)


def _candidates(field: Field) -> List[type]:
    """Concrete component subclasses of the field type, then every @factory
    registered for the type or any of its subclasses."""
    out = list(utils.generate_component_subclasses(field.type))
    for sub in utils.generate_subclasses(field.type):
        out.extend(FACTORY_REGISTRY.get(sub, ()))
    return out


def _resolve_class_name(value: Any, candidates: List[type]) -> Any:
    if not candidates or not isinstance(value, str):
        return value
    wanted = utils.convert_to_snake_case(value)
    for cls in candidates:
        if (
            value == cls.__name__
            or value == cls.__qualname__
            or wanted == utils.convert_to_snake_case(cls.__name__)
        ):
            return cls()
    return value


def _missing_component_error(full_name: str, type_label: str, candidates: List[type]):
    if candidates:
        listing = "\n    ".join([""] + [utils.type_name_str(c) for c in candidates])
        return ValueError(
            f"Component field '{full_name}' of type '{type_label}' has no default or "
            f"configured class. Please configure '{full_name}' with one of the "
            "following @component or @factory classes:" + listing
        )
    return ValueError(
        f"Component field '{full_name}' of type '{type_label}' has no default or "
        "configured class. No defined @component or @factory class satisfies this "
        f"type. Please define an @component class subclassing '{type_label}', or an "
        "@factory class with a `build()` method returning a "
        f"'{type_label}' instance. This class must be imported before invoking "
        "`configure()`."
    )


def _assign_field(instance: Any, field: Field, conf: Dict[str, Any], interactive: bool):
    """Decide the configured value (if any) of one field; returns nothing but
    records the value in ``instance``'s configured-values dict."""
    configured = instance.__dict__[_CONF_VALUES]
    in_scope = instance.__dict__[_IN_SCOPE]
    full_name = f"{instance.__component_name__}.{field.name}"
    is_cf = isinstance(field, ComponentField)
    candidates = _candidates(field) if is_cf else []

    if field.name in conf:
        value = conf.pop(field.name)
        if is_cf:
            value = _resolve_class_name(value, candidates)
        configured[field.name] = value
        _invalidate(instance, field.name)
    elif field.name in in_scope or field.allow_missing:
        pass
    elif is_cf and len(candidates) == 1:
        only = candidates[0]
        utils.warn(
            f"'{utils.type_name_str(only)}' is the only concrete component class that "
            f"satisfies the type of the annotated field '{full_name}'. Using an "
            "instance of this class by default."
        )
        configured[field.name] = only()
    elif interactive:
        if is_cf:
            if not candidates:
                raise ValueError(
                    "No component or factory class is defined which satisfies the type "
                    f"{_type_label(field.type)} of field {full_name}. If such a class "
                    "has been defined, it must be imported before calling `configure`."
                )
            configured[field.name] = utils.prompt_for_component_subclass(
                full_name, candidates
            )()
        else:
            configured[field.name] = utils.prompt_for_value(full_name, field.type)
    else:
        if is_cf:
            raise _missing_component_error(full_name, _type_label(field.type), candidates)
        raise ValueError(
            "No configuration value found for annotated field "
            f"'{full_name}' of type '{_type_label(field.type)}'."
        )
    in_scope.add(field.name)


def _check_leftover_keys(instance: Any, conf: Dict[str, Any]) -> None:
    fields = type(instance).__component_fields__
    for key in conf:
        head = key.split(".", 1)[0]
        ok = "." in key and isinstance(fields.get(head), ComponentField)
        if not ok:
            raise ValueError(
                f"Key '{key}' does not correspond to any field of component "
                f"'{instance.__component_name__}'." + _KEY_ERROR_HINT
            )


def configure(
    instance: Any,
    conf: Dict[str, Any],
    name: Optional[str] = None,
    interactive: bool = False,
) -> None:
    """Configure ``instance`` (and, recursively, its sub-components) from the
    flat dotted-key dict ``conf``.  Configured values take precedence over
    class defaults and ``__init__`` kwargs.  A component is configured once."""
    if not utils.is_component_instance(instance):
        raise TypeError(
            "Only @component, @factory, and @task instances can be configured. "
            f"Received: {instance}."
        )
    if instance.__component_configured__:
        raise ValueError(
            f"Component '{instance.__component_name__}' has already been configured."
        )
    if name is not None:
        instance.__component_name__ = name

    conf = dict(conf)
    fields = type(instance).__component_fields__
    for field in fields.values():
        _assign_field(instance, field, conf, interactive)
    _check_leftover_keys(instance, conf)

    for field in fields.values():
        if not isinstance(field, ComponentField):
            continue
        try:
            child = base_getattr(instance, field.name)
        except AttributeError:
            if field.allow_missing:
                continue
            raise
        if not utils.is_component_instance(child) or child.__component_configured__:
            continue
        child.__component_parent__ = instance
        child.__dict__[_IN_SCOPE] |= instance.__dict__[_IN_SCOPE]
        prefix = f"{field.name}."
        child_conf = {k[len(prefix):]: v for k, v in conf.items() if k.startswith(prefix)}
        configure(
            child,
            child_conf,
            name=f"{instance.__component_name__}.{field.name}",
            interactive=interactive,
        )

    instance.__component_configured__ = True
    if hasattr(type(instance), "__post_configure__"):
        instance.__post_configure__()
