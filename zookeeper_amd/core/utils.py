"""Small helpers shared by the component system.

Behavioural parity targets (reference file:line):

* ``missing`` sentinel ............ zookeeper/core/utils.py:11-16
* ``warn`` ........................ zookeeper/core/utils.py:19-20
* component / factory predicates .. zookeeper/core/utils.py:23-39
* subclass discovery .............. zookeeper/core/utils.py:42-57
* ancestor walk (scoping) ......... zookeeper/core/utils.py:60-74
* immutability / lazy wrapping .... zookeeper/core/utils.py:109-132
* naming + CLI value parsing ...... zookeeper/core/utils.py:135-160
* interactive prompts ............. zookeeper/core/utils.py:163-195

The type checker lives in :mod:`zookeeper_amd.core.typecheck` (the reference
delegates to ``typeguard``, which is not available in this image).
"""

from __future__ import annotations

import ast
import inspect
import re
from typing import Any, Callable, Iterator, Sequence, Type, TypeVar

import click

T = TypeVar("T")

# Attribute names used as markers on component classes.  Kept in one place so
# the predicates below and the decorators agree.
COMPONENT_MARKER = "__component_name__"
FACTORY_MARKER = "__component_factory_return_type__"


class Missing:
    """Sentinel type for "no value" (distinct from ``None``)."""

    _instance = None

    def __new__(cls):
        if cls._instance is None:
            cls._instance = super().__new__(cls)
        return cls._instance

    def __repr__(self) -> str:
        return "<missing>"

    def __reduce__(self):
        return (Missing, ())


missing = Missing()


def warn(message: str) -> None:
    """Print a yellow ``WARNING: ...`` line on stderr."""
    click.secho(f"WARNING: {message}", fg="yellow", err=True)


# --------------------------------------------------------------------------- #
# Predicates
# --------------------------------------------------------------------------- #


def is_component_class(cls: Any) -> bool:
    """True only for classes that were *themselves* decorated (undecorated
    subclasses of a component are not components)."""
    try:
        return inspect.isclass(cls) and COMPONENT_MARKER in vars(cls)
    except (AttributeError, TypeError):
        return False


def is_component_instance(obj: Any) -> bool:
    return is_component_class(type(obj))


def is_factory_class(cls: Any) -> bool:
    return is_component_class(cls) and hasattr(cls, FACTORY_MARKER)


def is_factory_instance(obj: Any) -> bool:
    return is_factory_class(type(obj))


# --------------------------------------------------------------------------- #
# Class-hierarchy walks
# --------------------------------------------------------------------------- #


def generate_subclasses(cls: Any) -> Iterator[Type]:
    """Depth-first walk of ``cls`` and all its (transitive) subclasses."""
    if not inspect.isclass(cls):
        return
    stack = [cls]
    while stack:
        current = stack.pop()
        yield current
        try:
            children = current.__subclasses__()
        except TypeError:  # e.g. `type` itself needs an argument
            children = type.__subclasses__(current)
        # Reverse so that the first-declared subclass is visited first.
        stack.extend(reversed(children))


def generate_component_subclasses(cls: Any) -> Iterator[Type]:
    """Concrete (non-abstract) component classes among ``cls``'s subclasses."""
    for sub in generate_subclasses(cls):
        if is_component_class(sub) and not inspect.isabstract(sub):
            yield sub


def generate_component_ancestors_with_field(
    instance: Any, field_name: str, include_instance: bool = False
) -> Iterator[Any]:
    """Yield, closest first, the component ancestors (optionally ``instance``
    itself) that declare a field called ``field_name``."""
    node = instance if include_instance else instance.__component_parent__
    while node is not None:
        if field_name in type(node).__component_fields__:
            yield node
        node = node.__component_parent__


# --------------------------------------------------------------------------- #
# Value helpers
# --------------------------------------------------------------------------- #

_IMMUTABLE_SCALARS = (int, float, bool, str, frozenset)


def _is_immutable_scalar(value: Any) -> bool:
    return value is None or isinstance(value, _IMMUTABLE_SCALARS)


def is_immutable(value: Any) -> bool:
    """None / int / float / bool / str / frozenset, or a flat tuple of those."""
    if _is_immutable_scalar(value):
        return True
    return isinstance(value, tuple) and all(_is_immutable_scalar(v) for v in value)


def wrap_in_callable(value: T) -> Callable[[], T]:
    return lambda: value


def type_name_str(tp: Any) -> str:
    """Human-readable name of a class (qualified when possible)."""
    try:
        for attr in ("__qualname__", "__name__"):
            if hasattr(tp, attr):
                return str(getattr(tp, attr))
        return str(tp)
    except Exception:
        return "<unknown type>"


_CAMEL_1 = re.compile(r"(.)([A-Z][a-z]+)")
_CAMEL_2 = re.compile(r"([a-z0-9])([A-Z])")
_MULTI_UNDERSCORE = re.compile(r"__+")


def convert_to_snake_case(name: str) -> str:
    """``FooBar`` / ``fooBar`` / ``Foo_Bar`` / ``foo_bar`` -> ``foo_bar``."""
    s = _CAMEL_1.sub(r"\1_\2", name)
    s = _CAMEL_2.sub(r"\1_\2", s)
    return _MULTI_UNDERSCORE.sub("_", s).lower()


def parse_value_from_string(string: str) -> Any:
    """Parse a CLI value as a Python literal, falling back to the raw string."""
    try:
        return ast.literal_eval(string)
    except (ValueError, SyntaxError):
        return str(string)
    except Exception:
        raise ValueError(f"Could not parse '{string}'.")


# --------------------------------------------------------------------------- #
# Interactive prompts (`-i` mode)
# --------------------------------------------------------------------------- #


def prompt_for_value(field_name: str, field_type: Any) -> Any:
    return click.prompt(
        f"\nNo value found for field '{field_name}' of type '{field_type}'. ",
        prompt_suffix="Please enter a value for this parameter:\n> ",
        value_proc=parse_value_from_string,
    )


def prompt_for_component_subclass(component_name: str, classes: Sequence[T]) -> T:
    by_name = {c.__qualname__: c for c in classes}
    ordered = sorted(by_name)

    def to_index(raw: str) -> int:
        try:
            idx = int(raw) - 1
        except ValueError:
            idx = -1
        if 0 <= idx < len(ordered):
            return idx
        raise click.UsageError(f"Please enter a number between 1 and {len(ordered)}.")

    menu = "\n".join(f"{i + 1})  {n}" for i, n in enumerate(ordered))
    idx = click.prompt(
        f"\nNo instance found for nested component '{component_name}'. Please choose "
        "from one of the following component subclasses to instantiate:\n" + menu,
        prompt_suffix="\n> ",
        value_proc=to_index,
    )
    return by_name[ordered[idx]]


def type_check(value: Any, expected_type: Any) -> bool:
    """Does ``value`` satisfy ``expected_type``?

    A @factory instance is checked through the return annotation of its
    ``build()`` (``issubclass``); when that comparison is impossible (typing
    generics) a warning is printed and the check passes.  Reference:
    zookeeper/core/utils.py:77-103.
    """
    from zookeeper_amd.core.typecheck import check_type

    if is_factory_instance(value):
        ret = getattr(type(value), FACTORY_MARKER)
        try:
            return issubclass(ret, expected_type)
        except TypeError:
            warn(f"Unable to check that {ret} is a sub-type of {expected_type}.")
            return True
    return check_type(value, expected_type)
