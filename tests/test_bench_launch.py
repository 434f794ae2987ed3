"""bench.py's rank launch: `bench.py --gpus N` must time N
ranks -- started by a launcher (torch.distributed.run: WORLD_SIZE set and equal
to N) or by bench.py itself (no launcher: N child processes, one per GPU, started
before anything touches the GPU) -- and must refuse a --gpus that differs from
the launcher's world size.  The reference counterpart is the sequential per-file
loop this shards (kf2vec/main.py:301)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _env(**kw):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "KF_BENCH_REHEARSE")}
    e.update(kw)
    return e


def test_resolve_world():
    import bench
    a = bench.parse_args([])
    assert bench.resolve_world(a, {}) == (1, False)
    assert bench.resolve_world(a, {"WORLD_SIZE": "4"}) == (4, False)       # torchrun without --gpus
    a = bench.parse_args(["--gpus", "8"])
    assert bench.resolve_world(a, {}) == (8, True)                          # spawn the 8 ranks here
    assert bench.resolve_world(a, {"WORLD_SIZE": "8"}) == (8, False)
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.resolve_world(a, {"WORLD_SIZE": "2"})
    with pytest.raises(SystemExit):
        bench.resolve_world(bench.parse_args(["--gpus", "0"]), {})


def test_gpus_mismatch_refused_before_any_gpu_work():
    """WORLD_SIZE=2 with --gpus 4: exit non-zero at once, with a message, and no
    JSON line (nothing was timed)."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=_env(WORLD_SIZE="2"),
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0
    assert "WORLD_SIZE=2" in p.stderr
    assert p.stdout.strip() == ""


def test_spawn_reports_failing_rank(tmp_path):
    """spawn_ranks relays rank 0's stdout and returns non-zero when a rank fails
    (here: every rank runs bench.py on a machine with no usable GPU, or a stub
    that fails rank 1 only)."""
    import bench
    stub = tmp_path / "stub.py"
    stub.write_text("import os, sys\n"
                    "r = int(os.environ['RANK'])\n"
                    "assert os.environ['WORLD_SIZE'] == '3' and os.environ['MASTER_ADDR'] == '127.0.0.1'\n"
                    "print('{\"rank\": %d}' % r) if r == 0 else None\n"
                    "sys.exit(3 if r == 1 else 0)\n")
    orig = bench.__file__
    try:
        bench.__file__ = str(stub)
        rc = bench.spawn_ranks(3, [], env=_env(KF_BENCH_REHEARSE="1"))
    finally:
        bench.__file__ = orig
    assert rc == 3


@pytest.mark.gpu
def test_bench_gpus2_spawns_two_ranks():
    """`python bench.py --gpus 2` with no launcher runs two ranks (both on cuda:0
    over gloo under KF_BENCH_REHEARSE=1 on a one-GPU box) over the configs[3]
    batch shape (64 genomes sharded g mod 2), parity ok, n_gpus 2, world size 2
    as torch.distributed reports it."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--total-genomes", "64",
           "--sub-batch", "16", "--seq-len", "300000", "--steps", "2", "--warmup", "1", "--no-cpu",
           "--e2e-genomes", "0", "--sparse-k", "0"]
    p = subprocess.run(cmd, env=_env(KF_BENCH_REHEARSE="1"), capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["ranks"]["world_size_reported"] == 2
    assert out["ranks"]["launcher"].startswith("bench.py --gpus")
    assert "BASELINE configs[3]" in out["config"]["workload"] and out["config"]["global_batch"] == 64
    assert out["parity"] == "ok"


@pytest.mark.gpu
def test_bench_rccl_collectives_one_rank():
    """The RCCL side of bench.py's multi-GPU path, which the driver's 8-GPU SCALE
    run is the first to execute with more than one GPU: init_process_group("nccl",
    device_id=...) as bench.main calls it, then Workload's own barrier, all_ok
    (float32 MAX) and max_over_ranks (float64 MAX) on device tensors, over a
    one-rank RCCL group (the methods run their collectives whenever world > 1)."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    code = "\n".join([
        "import os, sys, torch, torch.distributed as dist",
        f"sys.path.insert(0, {ROOT!r})",
        "import bench",
        f"os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT='{port}', RANK='0', WORLD_SIZE='1', LOCAL_RANK='0')",
        "torch.cuda.set_device(0)",
        "dist.init_process_group('nccl', device_id=torch.device('cuda', 0))",
        "W = bench.Workload.__new__(bench.Workload)",
        "W.torch, W.dev, W.world, W.dist, W.rehearse = torch, torch.device('cuda', 0), 2, dist, False",
        "W.barrier()",
        "assert W.all_ok(True) and not W.all_ok(False)",
        "assert W.max_over_ranks(1.5, 2.25) == (1.5, 2.25)",
        "assert dist.get_backend() == 'nccl'",
        "dist.destroy_process_group()",
        "print('rccl ok')",
    ])
    p = subprocess.run([sys.executable, "-c", code], env=_env(), capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and "rccl ok" in p.stdout, p.stderr[-3000:]
