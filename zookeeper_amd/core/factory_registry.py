"""Process-global registry of @factory classes keyed by ``build()``'s return
annotation (parity: zookeeper/core/factory_registry.py:8).

Values are insertion-ordered sets (a ``dict`` with ``None`` values) so that
candidate lists, and therefore error messages and name resolution, are
deterministic across runs.  ``cls in FACTORY_REGISTRY[T]`` works as for a set.
"""

from typing import Any, Dict, Type


class _OrderedClassSet(dict):
    def add(self, cls: Type) -> None:
        self[cls] = None

    def __repr__(self) -> str:
        return "{" + ", ".join(c.__qualname__ for c in self) + "}"


FACTORY_REGISTRY: Dict[Any, _OrderedClassSet] = {}


def register_factory(return_type: Any, cls: Type) -> None:
    FACTORY_REGISTRY.setdefault(return_type, _OrderedClassSet()).add(cls)
