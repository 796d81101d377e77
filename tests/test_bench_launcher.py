"""CPU: `bench.py --gpus N` starts its own one-rank-per-GPU launcher (torch.distributed.run as a
child process) when no launcher is around it, and refuses a world that differs from --gpus.
The rehearsal mode (--launch-check) rendezvous over gloo and all-reduces once, touching no GPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def test_self_launch_two_ranks_gloo():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--launch-check"], cwd=ROOT,
                       env=_env(STARK_BENCH_BACKEND="gloo"), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout            # rank 0 alone prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks_in_all_reduce"] == 2


def test_world_mismatch_is_refused():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--launch-check"], cwd=ROOT,
                       env=_env(WORLD_SIZE="2", RANK="0"), capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=2 but --gpus 4" in r.stderr


def test_single_gpu_runs_in_process():
    r = subprocess.run([sys.executable, "bench.py", "--launch-check"], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["n_gpus"] == 1
