"""Native RCCL DP module (csrc/dist/dist.cpp): the GPU-free parts on CPU (TCP bootstrap of the
ncclUniqueId blob across processes, shard ranges), the RCCL runner on the GPU (world 1 through the
fork launcher of apps/stereo_bench_dp.cpp; multi-GPU runs are the driver's)."""
import ctypes as C
import json
import multiprocessing as mp
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "stereoalgorithms_amd", "lib", "libstereo_dist.so")
BIN = os.path.join(ROOT, "stereoalgorithms_amd", "bin", "stereo_bench_dp")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _peer(rank, world, port, q, addr=b"127.0.0.1"):
    lib = C.CDLL(LIB, mode=C.RTLD_GLOBAL)
    buf = (C.c_ubyte * 128)()
    if rank == 0:
        for i in range(128):
            buf[i] = (i * 7 + 3) & 0xFF
    rc = lib.sa_dist_exchange_blob(rank, world, addr, port, buf, C.c_size_t(128), 20000)
    q.put((rank, rc, bytes(buf)))


@pytest.mark.skipif(not os.path.exists(LIB), reason="native build missing")
@pytest.mark.parametrize("world,addr", [(2, b"127.0.0.1"), (4, b"127.0.0.1"), (2, b"localhost")])
def test_unique_id_bootstrap_tcp(world, addr):
    """MASTER_ADDR as a dotted literal and as a hostname (torchrun passes socket.getfqdn())."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_peer, args=(r, world, port, q, addr)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (rc, b) for r, rc, b in (q.get(timeout=60) for _ in procs)}
    for p in procs:
        p.join(timeout=30)
    want = bytes((i * 7 + 3) & 0xFF for i in range(128))
    assert all(res[r][0] == 0 for r in range(world)), res
    assert all(res[r][1] == want for r in range(world))


@pytest.mark.skipif(not os.path.exists(LIB), reason="native build missing")
def test_bootstrap_times_out_without_rank0():
    lib = C.CDLL(LIB, mode=C.RTLD_GLOBAL)
    buf = (C.c_ubyte * 16)()
    assert lib.sa_dist_exchange_blob(1, 2, b"127.0.0.1", _free_port(), buf, C.c_size_t(16), 300) == -1


@pytest.mark.skipif(not os.path.exists(LIB), reason="native build missing")
def test_communicator_init_deadline_loop():
    """the communicator is created non-blocking (ncclCommInitRankConfig, blocking = 0) and its
    init / enqueues are polled through one deadline loop (settle): it returns 0 once the status reaches ncclSuccess,
    1 on an RCCL error, and -1 when the status is still ncclInProgress at SA_DIST_TIMEOUT -- a peer that never joins
    fails the job instead of hanging it.  Exercised on the CPU with a scripted status source (ncclInProgress = 7,
    ncclSuccess = 0, ncclSystemError = 2)."""
    import time
    lib = C.CDLL(LIB, mode=C.RTLD_GLOBAL)
    assert lib.sa_dist_settle_probe(0, 0, 1000) == 0
    assert lib.sa_dist_settle_probe(25, 0, 5000) == 0  # in progress for a while, then up
    assert lib.sa_dist_settle_probe(3, 2, 5000) == 1   # init failed
    t0 = time.perf_counter()
    assert lib.sa_dist_settle_probe(1 << 30, 0, 300) == -1  # never settles: the deadline ends it
    assert 0.25 < time.perf_counter() - t0 < 5.0


@pytest.mark.gpu
def test_native_dp_bench_world1():
    env = dict(os.environ, SA_DIST_TIMEOUT="120", SA_DP_GATHER_WORLD1="1")
    r = subprocess.run([BIN, "--nproc", "1", "--model", "raftstereo-realtime", "--batch", "2", "--steps", "3",
                        "--warmup", "1"], capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["n_gpus"] == 1 and rec["finite"] and rec["value"] > 0


@pytest.mark.gpu
def test_native_dp_bench_same_workload_as_bench_py(tmp_path):
    """stereo_bench_dp times bench.py's step -- per-step H2D of pinned host inputs on the copy
    stream, the frame graph with point-cloud reprojection, the gather path -- so at world 1 on the same box and with
    the same tactic plan (shared SA_PLAN_DIR) their ms/step agree (5 % here; the committed record is tighter)."""
    env = dict(os.environ, SA_DIST_TIMEOUT="120", SA_PLAN_DIR=str(tmp_path))
    env.pop("SA_DP_GATHER_WORLD1", None)
    args = ["--model", "raftstereo-realtime", "--steps", "30", "--warmup", "3"]
    r = subprocess.run([BIN, "--nproc", "1", "--batch", "8", *args], capture_output=True, text=True, timeout=200,
                       env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    nat = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--per-gpu-batch", "8", "--no-latency", *args],
                       capture_output=True, text=True, timeout=200, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    py = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    print(f"native {nat['ms_per_step']} ms/step vs bench.py {py['ms_per_step']} ms/step "
          f"(rank min/max {nat['rank_step_ms']} / {py['rank_step_ms']})")
    assert nat["finite"] and nat["plans_identical_across_ranks"]
    assert abs(nat["ms_per_step"] / py["ms_per_step"] - 1) < 0.05
