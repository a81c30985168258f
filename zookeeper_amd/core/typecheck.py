"""A self-contained runtime type checker for ``Field`` annotations.

The reference delegates to ``typeguard.check_type`` (zookeeper/core/utils.py:96-103,
typeguard 2.x semantics).  typeguard is not installed in this image and there
is no package index, so this module implements the subset of PEP 484 that
configuration values realistically use:

* plain classes (``isinstance``), with the PEP 484 numeric tower: an ``int``
  satisfies ``float`` and ``int``/``float`` satisfy ``complex`` (typeguard 2.x
  behaves the same way);
* ``Any`` / ``object`` / ``None``;
* ``Union`` / ``Optional`` / ``X | Y``;
* ``List`` / ``Sequence`` / ``Set`` / ``FrozenSet`` / ``Iterable`` /
  ``Collection`` and their PEP 585 spellings (every element is checked);
* ``Tuple[...]`` in its fixed-length, variadic (``Tuple[T, ...]``) and empty
  (``Tuple[()]``) forms;
* ``Dict`` / ``Mapping`` / ``MutableMapping`` (keys and values are checked);
* ``Type[T]``, ``Callable[...]`` (callability only), ``Literal[...]``,
  ``Annotated[T, ...]``, ``TypeVar`` (bound / constraints), ``NewType``;
* forward references (strings / ``ForwardRef``) cannot be resolved without the
  defining module's namespace and are accepted.

Anything else falls back to an ``isinstance`` check on the un-subscripted
origin when there is one, and is accepted otherwise.
"""

from __future__ import annotations

import collections
import collections.abc as cabc
import inspect
import types
import typing
from typing import Any, Tuple

__all__ = ["check_type"]

_NoneType = type(None)

# Origins whose arguments describe every element of an iterable container.
_ELEMENTWISE = {
    list,
    set,
    frozenset,
    cabc.Sequence,
    cabc.MutableSequence,
    cabc.Set,
    cabc.MutableSet,
    cabc.Iterable,
    cabc.Collection,
    cabc.Container,
    cabc.Reversible,
    collections.deque,
}
_MAPPINGS = {dict, cabc.Mapping, cabc.MutableMapping}
# Iterators/generators cannot be checked element-wise without consuming them.
_NO_ELEMENT_CHECK = {cabc.Iterator, cabc.Generator, cabc.AsyncIterator}


def _is_union(origin: Any) -> bool:
    if origin is typing.Union:
        return True
    union_type = getattr(types, "UnionType", None)
    return union_type is not None and origin is union_type


def _check_class(value: Any, cls: type) -> bool:
    if cls is float:
        return isinstance(value, (float, int))
    if cls is complex:
        return isinstance(value, (complex, float, int))
    try:
        return isinstance(value, cls)
    except TypeError:
        return True


_ORIGIN_ARGS: dict = {}


def _origin_args(expected: Any) -> Tuple[Any, Tuple[Any, ...]]:
    """``typing.get_origin`` / ``get_args``, memoised per annotation (the
    same few annotations are checked on every configure / first access)."""
    try:
        return _ORIGIN_ARGS[expected]
    except KeyError:
        pass
    except TypeError:  # unhashable annotation (e.g. Annotated metadata)
        return typing.get_origin(expected), typing.get_args(expected)
    r = (typing.get_origin(expected), typing.get_args(expected))
    _ORIGIN_ARGS[expected] = r
    return r


def check_type(value: Any, expected: Any) -> bool:  # noqa: C901 - a dispatcher
    """Return True if ``value`` satisfies the annotation ``expected``."""
    if type(expected) is type:  # a plain class (int, str, a component, ...)
        if expected is float:
            return isinstance(value, (float, int))
        if expected is complex:
            return isinstance(value, (complex, float, int))
        return isinstance(value, expected)
    if expected is Any or expected is object or expected is inspect.Parameter.empty:
        return True
    if expected is None or expected is _NoneType:
        return value is None
    if isinstance(expected, (str, typing.ForwardRef)):
        return True
    if isinstance(expected, typing.TypeVar):
        if expected.__bound__ is not None:
            return check_type(value, expected.__bound__)
        if expected.__constraints__:
            return any(check_type(value, c) for c in expected.__constraints__)
        return True
    # `typing.NewType` produces a function (3.9) or a NewType object (3.10+).
    supertype = getattr(expected, "__supertype__", None)
    if supertype is not None:
        return check_type(value, supertype)

    origin, args = _origin_args(expected)

    if origin is None:
        if inspect.isclass(expected):
            return _check_class(value, expected)
        if expected is typing.Callable:
            return callable(value)
        # Unknown typing construct (e.g. a bare special form): accept.
        return True

    if _is_union(origin):
        return any(check_type(value, a) for a in args)
    if origin is typing.Literal:
        return any(value == a and type(value) is type(a) for a in args)
    if origin is getattr(typing, "Annotated", object()) or (
        hasattr(expected, "__metadata__") and args
    ):
        return check_type(value, args[0])
    if origin is type:
        if not inspect.isclass(value):
            return False
        if not args or args[0] is Any:
            return True
        target = args[0]
        if _is_union(typing.get_origin(target)):
            return any(
                inspect.isclass(t) and issubclass(value, t) for t in typing.get_args(target)
            )
        if isinstance(target, typing.TypeVar):
            target = target.__bound__ or object
        try:
            return issubclass(value, target)
        except TypeError:
            return True
    if origin is cabc.Callable:
        return callable(value)
    if origin is tuple:
        if not isinstance(value, tuple):
            return False
        if not args:
            return True
        if len(args) == 2 and args[1] is Ellipsis:
            return all(check_type(v, args[0]) for v in value)
        if args == ((),):  # `Tuple[()]`
            return len(value) == 0
        if len(args) != len(value):
            return False
        return all(check_type(v, a) for v, a in zip(value, args))
    if origin in _MAPPINGS:
        if not _check_class(value, origin):
            return False
        if len(args) != 2:
            return True
        key_t, val_t = args
        return all(check_type(k, key_t) and check_type(v, val_t) for k, v in value.items())
    if origin in _ELEMENTWISE:
        if not _check_class(value, origin):
            return False
        if not args:
            return True
        return all(check_type(v, args[0]) for v in value)
    if origin in _NO_ELEMENT_CHECK:
        return _check_class(value, origin)

    # A parameterised user generic (e.g. `Foo[int]`): check the origin only.
    if inspect.isclass(origin):
        return _check_class(value, origin)
    return True
