"""The N-rank bench path on real hardware, rehearsed on one GPU: `bench.py --gpus 2` spawns
two rank processes (bitar_amd.launch), each drives the HIP engine on the box's GPU, the
size all-gather runs over gloo on host copies (BITAR_DIST_BACKEND=gloo; RCCL refuses two
ranks on one device), and rank 0 prints the one JSON line.  The 8-GPU RCCL run is the
driver's; this covers the launcher, per-rank device work, barriers, max-over-ranks timing
and the sharded legs (headline, configs[3] record batch, Zstd, DEFLATE)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def test_bench_two_ranks_share_one_gpu():
    env = dict(os.environ, BITAR_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--bytes", str(64 << 20), "--record-bytes", str(256 << 20),
           "--only", "recordbatch,zstd,deflate"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["roundtrip_ok"] and r["value"] > 0
    assert r["config"]["segments_per_gpu"] == 1024  # 128 MiB job, batches of 256 segments
    # per-rank spread of the timed region and launch durations (min, max over ranks)
    sp = r["rank_spread"]
    assert sp["elapsed_s"][0] <= sp["elapsed_s"][1] and sp["elapsed_max_over_min"] >= 1.0
    assert sp["compress_launch_ms"][0] <= sp["compress_launch_ms"][1]
    for leg in ("recordbatch", "zstd", "deflate"):
        assert r[leg]["roundtrip_ok"], leg


def test_bench_one_rank_rccl_collectives():
    """The RCCL branches on one GPU: under torch.distributed.run with one rank, bench.py
    forms a one-rank "nccl" process group bound with device_id, the size all-gather runs
    dist.all_gather_into_tensor on device tensors (bitar_amd.dist.SizeGather's collective
    branch) and the max-over-ranks timing runs dist.all_reduce on device tensors
    (bench.reduce_max_sum) -- the code the 8-GPU run uses, at world size 1."""
    import socket
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "BITAR_DIST_BACKEND"):
        env.pop(k, None)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
           "--bytes", str(64 << 20), "--record-bytes", str(256 << 20),
           "--only", "recordbatch,zstd", "--no-cpu-baseline"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    r = json.loads(lines[0])
    assert r["n_gpus"] == 1 and r["roundtrip_ok"]
    assert "RCCL all-gather" in r["config"]["parallelism"], r["config"]
    assert "RCCL size all-gather" in r["recordbatch"]["workload"]
    assert r["recordbatch"]["roundtrip_ok"] and r["zstd"]["roundtrip_ok"]
