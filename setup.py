"""pip-installable package (reference counterpart: setup.py:1-22 of the
`kfac` package).  `pip install .` (or `python setup.py build_ext --inplace`)
compiles every csrc/*.hip for gfx950 with hipcc into
distributed_kfac_pytorch_amd/_native/libkfac_hip.so (csrc/build.py) and ships
it inside the package; the Python side loads it with ctypes
(ops/_lib.py).  Without hipcc (a CPU-only machine) the package installs
without the native library and runs the torch reference paths."""
import importlib.util
import os
import shutil

from setuptools import find_packages, setup
from setuptools.command.build_ext import build_ext
from setuptools.command.build_py import build_py

ROOT = os.path.dirname(os.path.abspath(__file__))
LIB_REL = os.path.join('distributed_kfac_pytorch_amd', '_native', 'libkfac_hip.so')


def _build_native():
    spec = importlib.util.spec_from_file_location('kfac_csrc_build',
                                                  os.path.join(ROOT, 'csrc', 'build.py'))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    hipcc = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
    if not (os.path.exists(hipcc) or shutil.which('hipcc')):
        print('hipcc not found: installing without the gfx950 library (torch reference paths)')
        return False
    mod.build()
    return True


class BuildHip(build_ext):
    """build_ext: the HIP library (in place, next to the Python sources)."""

    def run(self):
        _build_native()


class BuildPy(build_py):
    """build_py: build the HIP library first so it is copied with the package."""

    def run(self):
        _build_native()
        super().run()
        src = os.path.join(ROOT, LIB_REL)
        if os.path.exists(src):
            dst = os.path.join(self.build_lib, LIB_REL)
            os.makedirs(os.path.dirname(dst), exist_ok=True)
            shutil.copy2(src, dst)


def _version():
    with open(os.path.join(ROOT, 'distributed_kfac_pytorch_amd', '__init__.py')) as f:
        for line in f:
            if line.startswith('__version__'):
                return line.split('=')[1].strip().strip("'\"")
    return '0.0.0'


setup(
    name='distributed_kfac_pytorch_amd',
    version=_version(),
    description='MI355X-native distributed K-FAC preconditioner for PyTorch-ROCm '
                '(hand-written gfx950 HIP kernels, RCCL over xGMI)',
    packages=find_packages(include=['distributed_kfac_pytorch_amd',
                                    'distributed_kfac_pytorch_amd.*']),
    package_data={'distributed_kfac_pytorch_amd': ['_native/*.so']},
    python_requires='>=3.8',
    install_requires=['torch'],
    cmdclass={'build_ext': BuildHip, 'build_py': BuildPy},
    zip_safe=False,
)
