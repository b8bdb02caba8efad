import faulthandler
import os
import sys
import traceback

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# Every test announces itself on the real stderr before it runs and a failing
# test prints its node id, exception and innermost frames before pytest builds
# its long report.  A process that dies afterwards (abort, GPU fault) still
# leaves the name of the test and the failure in the tail of the log.
_MARK = os.environ.get('KFAC_TEST_MARKERS', '1') != '0'


def _emit(msg):
    try:
        sys.__stderr__.write(msg + '\n')
        sys.__stderr__.flush()
    except Exception:
        pass


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP) device')
    config.addinivalue_line('markers', 'slow: long-running test')


@pytest.hookimpl(trylast=True)
def pytest_sessionstart(session):
    # Keep a fatal-signal dump short (the current thread only) so the test
    # markers printed just before it stay inside a log tail.
    if _MARK and faulthandler.is_enabled():
        try:
            faulthandler.enable(file=sys.__stderr__, all_threads=False)
        except Exception:
            pass


def pytest_runtest_logstart(nodeid, location):
    if _MARK:
        _emit('[kfac-test] START %s' % nodeid)


def pytest_runtest_logfinish(nodeid, location):
    if _MARK:
        _emit('[kfac-test] END %s' % nodeid)


@pytest.hookimpl(tryfirst=True, hookwrapper=True)
def pytest_runtest_makereport(item, call):
    if _MARK and call.excinfo is not None and call.when in ('setup', 'call', 'teardown') \
            and not call.excinfo.errisinstance(pytest.skip.Exception):
        ex = call.excinfo
        try:
            frames = traceback.extract_tb(ex.tb)[-4:]
            where = ' <- '.join('%s:%d %s' % (os.path.basename(f.filename), f.lineno, f.name)
                                for f in reversed(frames))
            _emit('[kfac-test] FAILED(%s) %s: %s\n[kfac-test]   at %s'
                  % (call.when, item.nodeid, ex.exconly()[:2000], where))
        except Exception:
            _emit('[kfac-test] FAILED(%s) %s' % (call.when, item.nodeid))
    yield


@pytest.fixture(autouse=True)
def _reset_comm():
    from distributed_kfac_pytorch_amd import comm
    comm.reset_comm_backend()
    yield
    comm.reset_comm_backend()


def gpu_available():
    import torch
    return torch.cuda.is_available()
