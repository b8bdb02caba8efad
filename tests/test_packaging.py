"""setup.py: metadata, package discovery and a wheel that carries the gfx950
library (built in-tree by csrc/build.py)."""
import glob
import os
import shutil
import subprocess
import sys
import zipfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_setup_metadata():
    out = subprocess.run([sys.executable, 'setup.py', '--name', '--version'], cwd=ROOT,
                         capture_output=True, text=True, check=True).stdout.split()
    import distributed_kfac_pytorch_amd as kfac
    assert out[-2:] == ['distributed_kfac_pytorch_amd', kfac.__version__]


def _drop_wheel_build_dirs():
    # setuptools stages the wheel in ROOT/build/{lib,bdist.*} and writes an
    # egg-info: generated copies of the package, removed so they are never
    # mistaken for sources (csrc/build.py's objects in build/hip stay)
    for d in glob.glob(os.path.join(ROOT, 'build', 'lib*')) + \
            glob.glob(os.path.join(ROOT, 'build', 'bdist*')) + \
            glob.glob(os.path.join(ROOT, '*.egg-info')):
        shutil.rmtree(d, ignore_errors=True)


def test_wheel_contains_package_and_native_lib(tmp_path):
    try:
        subprocess.run([sys.executable, '-m', 'pip', 'wheel', '--no-deps', '--no-build-isolation',
                        '-w', str(tmp_path), ROOT], check=True, capture_output=True, timeout=900)
    finally:
        _drop_wheel_build_dirs()
    wheels = [f for f in os.listdir(str(tmp_path)) if f.endswith('.whl')]
    assert len(wheels) == 1
    names = zipfile.ZipFile(os.path.join(str(tmp_path), wheels[0])).namelist()
    assert 'distributed_kfac_pytorch_amd/preconditioner.py' in names
    assert 'distributed_kfac_pytorch_amd/ops/_lib.py' in names
    if os.path.exists('/opt/rocm/bin/hipcc'):
        assert 'distributed_kfac_pytorch_amd/_native/libkfac_hip.so' in names
