"""pip-installable package: `pip install -e .` builds both native extensions
in-tree (csrc/build.py: g++ host runtime + hipcc gfx950 kernels) and exposes
the reference's two entry points as console scripts.

The Python package is imported as ``psx``; its sources live in
``parameter-server-architecture-on-apache-kafka_amd/`` (``psx`` is a symlink
to it for in-tree use).
"""
import os
import sys

from setuptools import setup
from setuptools.command.build_py import build_py

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = "parameter-server-architecture-on-apache-kafka_amd"


class BuildNative(build_py):
    """Compile _psx_host / _psx_hip before collecting package files."""

    def run(self):
        sys.path.insert(0, os.path.join(ROOT, "csrc"))
        import build as native_build  # csrc/build.py

        native_build.build_all(hip=os.environ.get("PSX_SKIP_HIP") != "1")
        super().run()


setup(
    name="psx-mi355x",
    version="0.1.0",
    description="MI355X-native parameter-server training engine (HIP/CDNA4 kernels, RCCL over xGMI)",
    python_requires=">=3.9",
    packages=["psx", "psx.apps", "psx.models", "psx.ops", "psx.parallel", "psx.runtime", "psx.utils"],
    package_dir={"psx": PKG_DIR, **{f"psx.{p}": f"{PKG_DIR}/{p}" for p in
                                     ("apps", "models", "ops", "parallel", "runtime", "utils")}},
    package_data={"psx": ["_psx_host*.so", "_psx_hip*.so"]},
    install_requires=["torch", "numpy", "pybind11"],
    entry_points={"console_scripts": [
        "psx-server=psx.apps.server_app_runner:main",
        "psx-worker=psx.apps.worker_app_runner:main",
    ]},
    cmdclass={"build_py": BuildNative},
)
