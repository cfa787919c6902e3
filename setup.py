"""Packaging for torchbooster_amd (reference packaging: /root/reference/setup.py:1-16).

``pip install .`` (or ``python setup.py build_ext --inplace``) compiles the gfx950
HIP/C++ library ``torchbooster_amd/_C.so`` through ``torchbooster_amd._build``
(hipcc --offload-arch=gfx950 + ninja, linked against the installed torch's HIP
runtime) and installs both ``torchbooster_amd`` and the ``torchbooster``
compatibility namespace, so scripts written against the reference import
unchanged.  Unlike the reference, the runtime requirements are declared.
"""
from __future__ import annotations

import shutil
from pathlib import Path

from setuptools import Extension, find_packages, setup
from setuptools.command.build_ext import build_ext

ROOT = Path(__file__).resolve().parent


class HipBuild(build_ext):
    """Delegates to the in-tree ninja build, then copies _C.so where setuptools expects it."""

    def run(self) -> None:
        if self.inplace:  # the in-tree torchbooster_amd/_C.so is the product; never shadow it
            self._ninja()
            return
        super().run()

    def _ninja(self) -> Path:
        import sys

        sys.path.insert(0, str(ROOT))
        from torchbooster_amd import _build

        return _build.build()

    def build_extension(self, ext: Extension) -> None:
        out = self._ninja()
        dest = Path(self.get_ext_fullpath(ext.name))
        dest.parent.mkdir(parents=True, exist_ok=True)
        if dest.resolve() != out.resolve():
            shutil.copy2(out, dest)


setup(
    name="torchbooster_amd",
    version="0.1.0",
    description="MI355X-native (gfx950 HIP + RCCL) re-implementation of TorchBooster",
    packages=find_packages(include=["torchbooster_amd", "torchbooster_amd.*", "torchbooster"]),
    package_data={"torchbooster_amd.ops": ["*.json", "*.csv"]},
    ext_modules=[Extension("torchbooster_amd._C", sources=[])],
    cmdclass={"build_ext": HipBuild},
    python_requires=">=3.8",
    install_requires=["torch", "numpy", "pyyaml"],
    extras_require={
        "huggingface_datasets": ["datasets"],
        "colored_logs": ["coloredlogs"],
    },
    zip_safe=False,
)
