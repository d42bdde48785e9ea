"""bench.py driver contract on CPU: torch.distributed.run with 1, 4 and 8 gloo ranks (8 = the
driver's scaling run on a full MI355X node, here on gloo).

The driver runs ``python -m torch.distributed.run --nproc-per-node N bench.py --gpus N``
on one node; this rehearses the same launch (gloo instead of RCCL, tiny net, torch
backend) and checks the single JSON line rank 0 prints: whole-job value, weak-scaling
global batch, and the ``dpN`` parallelism tag.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("nproc", [1, 4, 8])
def test_bench_json_line_under_torchrun(nproc):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", str(nproc), "--steps", "2", "--warmup", "1",
           "--backend", "torch", "--batch", "2", "--filters", "8", "--layers", "3", "--pool", "16",
           "--min-warmup-s", "0.5"]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1",
               PYTHONPATH=ROOT)
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    out = json.loads(lines[0])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config"):
        assert key in out
    assert out["n_gpus"] == nproc and out["steps"] == 2 and out["warmup"] == 1
    assert out["scaling"] == "weak" and out["higher_is_better"] is True
    assert out["config"]["global_batch"] == 2 * nproc
    assert out["config"]["parallelism"] == "dp%d" % nproc
    assert out["value"] > 0
    # diagnostics of the multi-rank run: live process group, per-rank step times, exposed all-reduce
    assert out["world_size"] == nproc and len(out["rank_ms_per_step"]) == nproc
    assert out["dist_backend"] == ("gloo" if nproc > 1 else "none")
    assert "allreduce_exposed_ms_per_step" in out
    assert out["data"].startswith("synthetic: ")  # teacher-labelled pool (learnable labels)
    # at least --warmup steps and at least --min-warmup-s seconds, same count on every rank
    assert out["warmup_steps_run"] >= 1 and (out["warmup_steps_run"] - 1) % 10 == 0 and out["warmup_s"] >= 0.5
    # value is the whole-job rate: global positions over the (max-over-ranks) timed span
    assert abs(out["value"] - 2 * nproc * 2 / (out["ms_per_step"] * 2 / 1e3)) / out["value"] < 0.01


def _plain_bench(extra, env_extra=None, timeout=600):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1", "--batch", "2",
           "--filters", "8", "--layers", "3", "--pool", "16", "--min-warmup-s", "0.5"] + extra
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1", PYTHONPATH=ROOT)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)


def test_bench_plain_launch_starts_the_ranks():
    """`python bench.py --gpus 4` with no torchrun: bench.py supervises 4 ranks itself and the one JSON
    line describes the 4-rank world (before round 6 it silently measured one rank)."""
    p = _plain_bench(["--gpus", "4", "--backend", "torch"])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 4 and out["world_size"] == 4 and out["dist_backend"] == "gloo"
    assert out["config"]["global_batch"] == 8 and out["config"]["parallelism"] == "dp4"
    assert len(out["rank_ms_per_step"]) == 4


def test_bench_refuses_world_mismatch():
    """--gpus 2 inside a 4-rank torchrun world is refused (non-zero exit, no JSON line)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--backend", "torch", "--batch", "2", "--filters", "8", "--layers", "3", "--pool", "16"]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1", PYTHONPATH=ROOT)
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode != 0
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert "WORLD_SIZE=4" in p.stderr


def test_bench_refuses_missing_gpus():
    """The HIP backend with --gpus 2 and no visible GPU exits 2 with a message instead of running."""
    p = _plain_bench(["--gpus", "2", "--backend", "hip"], timeout=300)
    assert p.returncode == 2, (p.returncode, p.stderr[-2000:])
    assert "GPU(s) are visible" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_bench_supervisor_forwards_sigterm(tmp_path):
    """A plain `bench.py --gpus 2` stopped with SIGTERM stops its ranks too (no orphaned rank processes)."""
    import signal
    import time

    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "torch", "--steps", "100000",
           "--warmup", "1", "--batch", "2", "--filters", "8", "--layers", "3", "--pool", "16", "--min-warmup-s", "0.5"]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1", PYTHONPATH=ROOT)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         start_new_session=True)
    time.sleep(25)  # ranks started and training
    pgid = os.getpgid(p.pid)
    p.send_signal(signal.SIGTERM)
    try:
        p.wait(timeout=60)
    finally:
        if p.poll() is None:
            os.killpg(pgid, signal.SIGKILL)
    assert p.returncode != 0
    time.sleep(2)
    # every process of the session (launcher + ranks) is gone
    alive = []
    for d in os.listdir("/proc"):
        if d.isdigit():
            try:
                if os.getpgid(int(d)) == pgid:
                    alive.append(int(d))
            except OSError:
                pass
    assert not alive, alive
