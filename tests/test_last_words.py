"""dpwa_last_words_set (include/dpwa_hip.h): the line registered is written once to its fd when the
process is ended by a signal or dies by one, the previous handler (faulthandler's, the default)
still runs after it, and a cleared line writes nothing.  bench.py registers its held result line
this way on rank 0, so torch.distributed.run stopping the job after another rank died, or an
abort inside the runtime, still leaves the measured line on stdout.  CPU only: the
library loads without a GPU."""
import os
import signal
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PRELUDE = """
import faulthandler, os, signal, sys, time
sys.path.insert(0, %r)
from dpwa_amd import _lib
_lib.load()
""" % ROOT


def _run(body):
    p = subprocess.run([sys.executable, "-c", PRELUDE + body], cwd=ROOT, capture_output=True, text=True, timeout=120)
    return p.returncode, p.stdout, p.stderr


def _lib_or_skip():
    sys.path.insert(0, ROOT)
    from dpwa_amd import _lib
    try:
        _lib.load()
    except _lib.DpwaLibraryError as e:
        pytest.skip(str(e))


@pytest.mark.parametrize("how,sig", [("os.kill(os.getpid(), signal.SIGTERM)", signal.SIGTERM),
                                     ("os.abort()", signal.SIGABRT),
                                     ("os.kill(os.getpid(), signal.SIGHUP)", signal.SIGHUP)])
def test_line_written_once_on_a_fatal_signal(how, sig):
    _lib_or_skip()
    rc, out, _ = _run("""
_lib.last_words(1, '{"first": 1}\\n')
_lib.last_words(1, '{"value": 2}\\n')
sys.stdout.flush()
%s
time.sleep(30)
""" % how)
    assert rc == -sig
    assert out == '{"value": 2}\n'


def test_cleared_line_writes_nothing():
    _lib_or_skip()
    rc, out, _ = _run("""
_lib.last_words(1, '{"value": 2}\\n')
_lib.last_words(1, '')
os.kill(os.getpid(), signal.SIGTERM)
time.sleep(30)
""")
    assert rc == -signal.SIGTERM and out == ""


def test_flush_writes_once_and_a_later_signal_writes_nothing():
    _lib_or_skip()
    rc, out, _ = _run("""
_lib.last_words(1, '{"value": 4}\\n')
assert _lib.last_words_flush() is True
assert _lib.last_words_flush() is False and _lib.last_words_written() is True
_lib.last_words(1, '{"value": 5}\\n')
assert _lib.last_words_flush() is False
os.kill(os.getpid(), signal.SIGTERM)
time.sleep(30)
""")
    assert rc == -signal.SIGTERM and out == '{"value": 4}\n'


def test_an_ignored_signal_stays_ignored():
    """SIGHUP ignored before (nohup): it neither writes the line nor ends the run."""
    _lib_or_skip()
    rc, out, _ = _run("""
signal.signal(signal.SIGHUP, signal.SIG_IGN)
_lib.last_words(1, '{"value": 6}\\n')
os.kill(os.getpid(), signal.SIGHUP)
time.sleep(0.2)
assert _lib.last_words_written() is False
assert _lib.last_words_flush() is True
""")
    assert rc == 0 and out == '{"value": 6}\n'


def test_previous_handler_still_runs():
    """faulthandler registered before (as bench.py does for SIGTERM) still dumps the threads."""
    _lib_or_skip()
    rc, out, err = _run("""
faulthandler.register(signal.SIGTERM, all_threads=True, chain=True)
_lib.last_words(1, '{"value": 3}\\n')
os.kill(os.getpid(), signal.SIGTERM)
time.sleep(30)
""")
    assert rc == -signal.SIGTERM and out == '{"value": 3}\n'
    assert "most recent call first" in err


def test_written_flag_and_bad_arguments():
    _lib_or_skip()
    from dpwa_amd import _lib
    assert _lib.last_words_written() is False
    with pytest.raises(_lib.DpwaError):
        _lib.call("dpwa_last_words_set", 1, b"x" * 20000, 20000)
    with pytest.raises(_lib.DpwaError):
        _lib.call("dpwa_last_words_set", -1, b"x", 1)
