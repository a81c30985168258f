"""Configuration / dependency-injection core (pure Python, no torch import).

Re-design of zookeeper/core (reference ``zookeeper/core/__init__.py:1-17``).
"""

from zookeeper_amd.core.cli import cli
from zookeeper_amd.core.component import base_getattr, component, configure
from zookeeper_amd.core.factory import factory
from zookeeper_amd.core.field import ComponentField, Field
from zookeeper_amd.core.partial_component import PartialComponent
from zookeeper_amd.core.task import task

__all__ = [
    "base_getattr",
    "cli",
    "component",
    "ComponentField",
    "configure",
    "factory",
    "Field",
    "PartialComponent",
    "task",
]
