"""CPU: the host worker pool of libstark_hip (csrc/host_pool.cpp: host_parallel, HostTask) runs every
item of every call exactly once before the call returns, with interleaved small and large calls from two
caller threads and from the side thread (the call mix of a rank process: 7-task staged uploads, 16-task
JSON renders, min(16, .)-task path checks).  The round-4 pool it replaced, restated in
tests/host_pool/pool_check.cpp, is the counter-example: its shared claim counter lets a worker leaving
call k run an item of call k + 1 (hazard 5), which this harness shows as an item run twice
or never, and ThreadSanitizer flags as a data race.  Sanitizers run on the host build only."""
import os
import subprocess

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "host_pool")


@pytest.fixture(scope="module")
def built():
    subprocess.run(["make", "-s", "-C", HERE], check=True, timeout=300)
    return HERE


def _run(prog, mode, calls, tsan=False):
    env = dict(os.environ)
    if tsan:
        env["TSAN_OPTIONS"] = "halt_on_error=1 exitcode=66"
    return subprocess.run([os.path.join(HERE, prog), mode, str(calls)], capture_output=True, text=True,
                          timeout=240, env=env)


def test_product_pool_exactly_once(built):
    r = _run("pool_check", "product", 600)
    assert r.returncode == 0, r.stderr


def test_round4_pool_fails_exactly_once(built):
    """The counter-example: the same harness catches the round-4 handoff (an item run twice or never, or
    a call that never returns, which the harness's watchdog reports; a stale worker may then also crash
    the process, which counts as the same failure)."""
    r = _run("pool_check", "r4", 600)
    assert r.returncode != 0, (r.returncode, r.stdout, r.stderr)
    assert "hits:" in r.stderr


def test_product_pool_tsan_clean(built):
    r = _run("pool_check_tsan", "product", 150, tsan=True)
    if "unexpected memory mapping" in r.stderr or "FATAL: ThreadSanitizer" in r.stderr:
        pytest.skip("ThreadSanitizer cannot run in this environment: " + r.stderr.strip().splitlines()[0])
    assert r.returncode == 0, r.stderr[-3000:]


def test_round4_pool_tsan_race(built):
    r = _run("pool_check_tsan", "r4", 150, tsan=True)
    if "unexpected memory mapping" in r.stderr or "FATAL: ThreadSanitizer" in r.stderr:
        pytest.skip("ThreadSanitizer cannot run in this environment")
    assert r.returncode != 0, (r.returncode, r.stderr[-2000:])
    assert "data race" in r.stderr or "hits:" in r.stderr
