"""CPU: the record walk split over host threads (csrc/host_walk.cpp, RecordWalk) equals the serial walk
(walk_records_into, the walk r1cs_trace_device and the verifier's circuit build used alone before) on
generated constraint sections: the same status, and on success the same factor offsets, counts and slot
bases.  The sections cover canonical, small-integer, -1 and zero coefficients (small integers and zeros are
the hard case for a part's guessed start), trailing bytes after the section, truncations, corrupted counts
and an over-claimed constraint count; each is walked in 2..16 parts, through the pool and in reverse order.
The harness also requires the split to hold on canonical coefficients (no serial fallback).  Plain and under
ThreadSanitizer (host code only)."""
import os
import subprocess

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "host_walk")


@pytest.fixture(scope="module")
def built():
    subprocess.run(["make", "-s", "-C", HERE], check=True, timeout=300)
    return HERE


def test_split_walk_equals_serial(built):
    r = subprocess.run([os.path.join(HERE, "walk_check"), "check", "4"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout, r.stderr)
    assert "all equal" in r.stdout


def test_split_walk_tsan(built):
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    r = subprocess.run([os.path.join(HERE, "walk_check_tsan"), "check", "1"], capture_output=True, text=True,
                       timeout=240, env=env)
    assert r.returncode == 0, (r.stdout, r.stderr)
