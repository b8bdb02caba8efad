"""Build the gfx950 HIP kernel library in-tree.

    python csrc/build.py [--force] [--jobs N]

Compiles every csrc/*.hip with `hipcc --offload-arch=gfx950` into object
files under build/, links them into
`distributed_kfac_pytorch_amd/_native/libkfac_hip.so` (plain C ABI, loaded
through ctypes by ops/_lib.py; no torch headers, no hipify).  Rebuilds only
when a source or header is newer than the library.
"""
import argparse
import concurrent.futures
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, 'csrc')
OUT_DIR = os.path.join(ROOT, 'distributed_kfac_pytorch_amd', '_native')
LIB = os.path.join(OUT_DIR, 'libkfac_hip.so')
BUILD = os.path.join(ROOT, 'build', 'hip')
ARCH = os.environ.get('KFAC_HIP_ARCH', 'gfx950')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
# kernarg preload: the first kernel arguments arrive in SGPRs, so a latency-
# bound launch does not start with a scalar load round trip
FLAGS = ['-O3', '-std=c++17', '-fPIC', '--offload-arch=' + ARCH, '-munsafe-fp-atomics',
         '-Wno-unused-result', '-mllvm', '-amdgpu-kernarg-preload-count=16']


# no vendor math library: every kernel is hand-written (the HIP runtime only)
LIBS = []


# The two-stage eigensolver (dense -> band -> tridiagonal, round 4) loses to
# the one-stage path on every routing measured (profiles/r5_eig_two_stage_
# mid_routing.log); it is built only on request: KFAC_BUILD_TWO_STAGE=1.
TWO_STAGE_SOURCES = ('eig_sy2sb.hip', 'eig_sb2st.hip', 'eig_q2.hip')


def two_stage_enabled():
    return os.environ.get('KFAC_BUILD_TWO_STAGE') == '1'


def sources():
    srcs = sorted(glob.glob(os.path.join(CSRC, '*.hip')))
    if not two_stage_enabled():
        srcs = [s for s in srcs if os.path.basename(s) not in TWO_STAGE_SOURCES]
    return srcs


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src):
    obj = os.path.join(BUILD, os.path.basename(src) + '.o')
    headers = glob.glob(os.path.join(CSRC, '*.h'))
    if _stale(obj, [src] + headers):
        cmd = [HIPCC] + FLAGS + ['-I', CSRC, '-c', src, '-o', obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError('hipcc failed for {}:\n{}\n{}'.format(src, ' '.join(cmd), r.stderr))
    return obj


def compile_optional():
    """Compile (not link) the opt-in sources, so every .hip stays buildable."""
    os.makedirs(BUILD, exist_ok=True)
    return [_compile(os.path.join(CSRC, f)) for f in TWO_STAGE_SOURCES]


def build(force=False, jobs=None, verbose=True):
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(OUT_DIR, exist_ok=True)
    srcs = sources()
    deps = srcs + glob.glob(os.path.join(CSRC, '*.h'))
    stamp = LIB + '.sources'
    listing = '\n'.join(os.path.basename(x) for x in srcs)
    same_set = os.path.exists(stamp) and open(stamp).read() == listing
    if not force and same_set and not _stale(LIB, deps):
        return LIB
    if force:
        for o in glob.glob(os.path.join(BUILD, '*.o')):
            os.remove(o)
    jobs = jobs or min(8, len(srcs))
    with concurrent.futures.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(_compile, srcs))
    tmp = LIB + '.tmp'
    cmd = [HIPCC, '--offload-arch=' + ARCH, '-shared', '-fPIC', '-o', tmp] + objs + LIBS
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError('link failed:\n{}\n{}'.format(' '.join(cmd), r.stderr))
    os.replace(tmp, LIB)
    with open(stamp, 'w') as f:
        f.write(listing)
    if verbose:
        print('built', LIB, 'from', len(objs), 'sources for', ARCH)
    return LIB


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--force', action='store_true')
    ap.add_argument('--jobs', type=int, default=None)
    a = ap.parse_args()
    try:
        build(force=a.force, jobs=a.jobs)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
