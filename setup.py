"""Install torcheval_amd and build its native extension (HIP kernels for gfx950 + host C++).

    pip install -e .                       # builds torcheval_amd/_C.so in-tree first
    TORCHEVAL_AMD_NIGHTLY=1 pip install .  # nightly package name + date version

The extension build is the same incremental hipcc / g++ driver as
``python -m torcheval_amd.ops.build`` (csrc/ -> build/native/ -> torcheval_amd/_C.so).
"""

import datetime
import os
import re

from setuptools import find_packages, setup
from setuptools.command.build_py import build_py
from setuptools.command.develop import develop

HERE = os.path.dirname(os.path.abspath(__file__))


def _version() -> str:
    with open(os.path.join(HERE, "torcheval_amd", "version.py")) as f:
        return re.search(r'__version__\s*=\s*"([^"]+)"', f.read()).group(1)


def _build_native() -> None:
    if os.environ.get("TORCHEVAL_AMD_SKIP_NATIVE") == "1":
        return
    import importlib.util

    spec = importlib.util.spec_from_file_location(
        "_tea_build", os.path.join(HERE, "torcheval_amd", "ops", "build.py")
    )
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.build()


class BuildPyWithNative(build_py):
    def run(self):
        _build_native()
        super().run()


class DevelopWithNative(develop):
    def run(self):
        _build_native()
        super().run()


nightly = os.environ.get("TORCHEVAL_AMD_NIGHTLY") == "1"
name = "torcheval-amd-nightly" if nightly else "torcheval-amd"
version = _version() + (datetime.date.today().strftime(".dev%Y%m%d") if nightly else "")

setup(
    name=name,
    version=version,
    description="MI355X-native (gfx950) model-evaluation metrics: torcheval API, HIP kernels, RCCL sync",
    long_description=open(os.path.join(HERE, "README.md")).read(),
    long_description_content_type="text/markdown",
    packages=find_packages(exclude=("tests", "tests.*", "examples", "benchmarks")),
    package_data={"torcheval_amd": ["_C.so"]},
    python_requires=">=3.9",
    install_requires=["torch", "numpy"],
    cmdclass={"build_py": BuildPyWithNative, "develop": DevelopWithNative},
)
