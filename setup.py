"""setuptools hook: build the gfx950 extension in-tree with hipcc before packaging.

``pip install -e .`` / ``python setup.py build_ext --inplace`` both run
pytorch_distributed_training_tutorials_amd/_build.py (hipcc --offload-arch=gfx950,
PYTORCH_ROCM_ARCH ignored: this framework targets MI355X only).
"""
import os
import sys

from setuptools import setup
from setuptools.command.build_ext import build_ext
from setuptools.command.build_py import build_py


def _build_native():
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from pytorch_distributed_training_tutorials_amd import _build

    _build.build()


class BuildExt(build_ext):
    def run(self):
        _build_native()


class BuildPy(build_py):
    def run(self):
        _build_native()
        super().run()


setup(cmdclass={"build_ext": BuildExt, "build_py": BuildPy})
