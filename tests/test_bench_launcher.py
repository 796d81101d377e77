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


def test_distributed_roofline_fields():
    """The N > 1 line's roofline (bench.py distributed_roofline): the local kernels' 2 x 64 B per shard
    element against HBM and the all-to-all's (G-1)/G x 32 B per element against G-1 xGMI links, from
    the phase times; nothing taken from the 1-GPU profiles."""
    sys.path.insert(0, ROOT)
    import bench
    n, world = 1 << 24, 8
    ph = {"local_ms": 1.5, "exchange_ms": 0.5, "finish_ms": 0.25}
    r = bench.distributed_roofline(ph, n, world, 24, [8, 8, 8], on_gloo=False)
    assert r["bound"] == "hbm" and r["traffic"] is None and r["phases_ms"] == ph
    assert abs(r["achieved"] - 128.0 * n / 1.75e-3 / 1e9) < 0.01
    x = r["exchange"]
    assert x["bytes_per_rank"] == 7 / 8 * n * 32 and x["peak"] == 7 * bench.XGMI_LINK_GBS
    assert abs(x["achieved"] - x["bytes_per_rank"] / 0.5e-3 / 1e9) < 0.01
    assert "xGMI" in x["bound"]
    assert "not an xGMI figure" in bench.distributed_roofline(ph, n, 2, 24, [8, 8, 8], on_gloo=True)["exchange"]["bound"]
