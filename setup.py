"""Packaging for zookeeper_amd (reference: setup.py:1-54).

``pip install .`` (or ``python setup.py build_ext --inplace``) compiles the
HIP kernels and C++ runtime with ``zookeeper_amd/csrc/build.py`` (hipcc,
``--offload-arch=gfx950``) into ``zookeeper_amd/_zkamd.so`` and ships it as
package data.  The library is a plain C-ABI shared object loaded with
ctypes, so there is no Python extension module to link against a specific
interpreter.  Set ``ZK_SKIP_NATIVE=1`` to package the pure-Python parts only
(config system, data, CPU paths).
"""

import os

from setuptools import Command, find_packages, setup
from setuptools.command.build_py import build_py

ROOT = os.path.dirname(os.path.abspath(__file__))


def _version() -> str:
    ns = {}
    with open(os.path.join(ROOT, "zookeeper_amd", "__init__.py")) as f:
        for line in f:
            if line.startswith("__version__ = \""):
                exec(line, ns)
                break
    return ns["__version__"]


class BuildNative(Command):
    """Compile the gfx950 library in-tree (``python setup.py build_native``)."""

    description = "compile HIP kernels + C++ runtime into zookeeper_amd/_zkamd.so"
    user_options = [("force", "f", "rebuild every object")]

    def initialize_options(self):
        self.force = 0

    def finalize_options(self):
        pass

    def run(self):
        if os.environ.get("ZK_SKIP_NATIVE") == "1":
            return
        import sys

        sys.path.insert(0, ROOT)
        from zookeeper_amd.csrc.build import build

        build(force=bool(self.force))


class BuildPyWithNative(build_py):
    def run(self):
        self.run_command("build_native")
        super().run()


setup(
    name="zookeeper_amd",
    version=_version(),
    description="Component-based experiment configuration with a native MI355X training runtime",
    long_description=open(os.path.join(ROOT, "README.md")).read(),
    long_description_content_type="text/markdown",
    license="Apache-2.0",
    packages=find_packages(include=["zookeeper_amd", "zookeeper_amd.*"]),
    package_data={"zookeeper_amd": ["_zkamd.so", "csrc/*.h", "csrc/kernels/*.hip",
                                    "csrc/kernels/*.h", "csrc/runtime/*.cpp"]},
    python_requires=">=3.8",
    install_requires=["click>=7.0", "torch>=2.1"],
    extras_require={"test": ["pytest>=6", "pytest-timeout"],
                    "data": ["datasets", "numpy"]},
    cmdclass={"build_native": BuildNative, "build_py": BuildPyWithNative},
    classifiers=[
        "Programming Language :: Python :: 3",
        "License :: OSI Approved :: Apache Software License",
        "Operating System :: POSIX :: Linux",
        "Topic :: Scientific/Engineering :: Artificial Intelligence",
    ],
)
