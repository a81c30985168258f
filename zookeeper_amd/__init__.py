"""zookeeper_amd — an MI355X-native experiment framework with zookeeper's
component / factory / task configuration API.

Public API (parity with reference ``zookeeper/__init__.py:1-29``)::

    from zookeeper_amd import (cli, component, ComponentField, configure,
                               factory, Field, PartialComponent, task)

Heavier subsystems (torch, HIP kernels, RCCL) live in sub-packages and are
imported lazily: ``zookeeper_amd.data``, ``zookeeper_amd.models``,
``zookeeper_amd.ops``, ``zookeeper_amd.nn``, ``zookeeper_amd.parallel``,
``zookeeper_amd.train``, ``zookeeper_amd.sweep``.
"""

from zookeeper_amd.core import (
    ComponentField,
    Field,
    PartialComponent,
    cli,
    component,
    configure,
    factory,
    task,
)

__version__ = "0.1.0"


def _installed_version() -> str:
    # Unlike the reference (zookeeper/__init__.py:12-18), an uninstalled source
    # checkout must still import: fall back to the in-tree version string.
    try:
        from importlib import metadata

        return metadata.version("zookeeper_amd")
    except Exception:
        return __version__


__version__ = _installed_version()

__all__ = [
    "cli",
    "ComponentField",
    "component",
    "configure",
    "factory",
    "Field",
    "PartialComponent",
    "task",
]
