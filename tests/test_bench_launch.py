"""bench.py's two N > 1 entry modes end to end on CPU, with --dry-backend gloo.

The driver may start the multi-GPU bench either as ``torch.distributed.run --nproc-per-node N
bench.py --gpus N`` or as a plain ``python bench.py --gpus N``.  In the plain mode bench.py starts
the N ranks itself (bench.launch_ranks) before anything touches a GPU.  Here both modes run with
N = 2 over gloo; the dry backend replaces the device batch with the library's host crc32c::Value
and the RCCL gather with torch.distributed.gather (no GPU).  Each run must print exactly one JSON
line (rank 0 only) with n_gpus = 2, two ranks in the group, every rank's self-check clean, and the
CRCs rank 0 gathered equal to the oracle's for the whole 2-shard batch, in record order
(per-record independence: karma-store/segment_file.cc:22, wal.cc:60).
"""
import hashlib
import json
import os
import socket
import subprocess
import sys

import oracle_lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
N_REC, REC = 1500, 256
ARGS = ["--gpus", "2", "--dry-backend", "gloo", "--steps", "3", "--warmup", "1", "--records-per-gpu", str(N_REC),
        "--rec-bytes", str(REC), "--prewarm-ms", "0", "--no-cpu-baseline"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env["OMP_NUM_THREADS"] = "1"
    return env


def _json_lines(out: str):
    return [json.loads(s) for s in out.splitlines() if s.startswith("{")]


def _check_line(line, launcher, n=2):
    assert line["n_gpus"] == n and line["dry_nranks"] == n and line["dry_backend"] == "gloo"
    assert line["launched_by"] == launcher
    assert line["self_check"]["mismatches"] == 0 and line["self_check"]["gather_mismatches"] == 0
    assert [p["mismatches"] for p in line["per_rank"]["self_check"]] == [0] * n
    want = oracle_lib.splitmix_fixed_crcs(42, REC, 0, n * N_REC)
    assert line["gathered_crcs"] == n * N_REC
    assert line["gathered_sha256_16"] == hashlib.sha256(want.astype("<u4").tobytes()).hexdigest()[:16]
    assert line["steps"] == 3 and line["value"] > 0


def test_plain_command_launches_its_own_ranks():
    """`python bench.py --gpus 2`: bench.py starts both ranks and prints one line."""
    r = subprocess.run([sys.executable, BENCH] + ARGS, cwd=ROOT, env=_env(), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    _check_line(lines[0], "bench.py")


def test_plain_command_four_ranks():
    """`python bench.py --gpus 4`: four self-launched ranks, every shard in the gathered CRCs."""
    args = [a if a != "2" else "4" for a in ARGS]
    r = subprocess.run([sys.executable, BENCH] + args, cwd=ROOT, env=_env(), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    _check_line(lines[0], "bench.py", n=4)


def test_torch_distributed_run_launch():
    """`torch.distributed.run --nproc-per-node 2 bench.py --gpus 2`: the outer launcher's ranks."""
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), BENCH] + ARGS,
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    _check_line(lines[0], "external")


def test_plain_command_failed_rank_ends_the_others():
    """A rank that fails before joining the group: the launcher ends the rank left waiting in
    init_process_group and exits with the failed rank's status (3), not 0 and not the status of
    the rank it terminated."""
    r = subprocess.run([sys.executable, BENCH] + ARGS + ["--dry-fail-rank", "1"], cwd=ROOT,
                       env=dict(_env(), KARMA_BENCH_GRACE_S="2"), capture_output=True, text=True, timeout=300)
    assert r.returncode == 3, (r.returncode, r.stderr[-3000:])
    assert _json_lines(r.stdout) == []


def test_single_rank_dry_line():
    """--gpus 1 stays a single process (no launcher) and prints the same line shape."""
    r = subprocess.run([sys.executable, BENCH] + [a if a != "2" else "1" for a in ARGS], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    (line,) = _json_lines(r.stdout)
    assert line["n_gpus"] == 1 and line["launched_by"] == "external" and line["self_check"]["mismatches"] == 0
    want = oracle_lib.splitmix_fixed_crcs(42, REC, 0, N_REC)
    assert line["gathered_sha256_16"] == hashlib.sha256(want.astype("<u4").tobytes()).hexdigest()[:16]


def test_plain_command_stop_signal_reaches_the_ranks():
    """SIGTERM to a self-launching bench.py (a driver's time limit) ends its ranks too: no rank is
    left running, holding a GPU, after the launcher has gone."""
    import signal
    import time

    import psutil
    args = [a if a != "3" else "100000" for a in ARGS]  # --steps 100000: the ranks keep running
    p = subprocess.Popen([sys.executable, BENCH] + args, cwd=ROOT, env=_env(), stdout=subprocess.DEVNULL,
                         stderr=subprocess.DEVNULL)
    try:
        t0 = time.time()
        kids = []
        while time.time() - t0 < 120:
            kids = psutil.Process(p.pid).children()
            if len(kids) == 2:
                break
            time.sleep(0.2)
        assert len(kids) == 2, kids
        time.sleep(3)  # the ranks are in their timed loop
        assert all(k.is_running() for k in kids)
        p.send_signal(signal.SIGTERM)
        assert p.wait(60) == 128 + signal.SIGTERM
        gone, alive = psutil.wait_procs(kids, timeout=30)
        assert not alive, alive
    finally:
        if p.poll() is None:
            p.kill()
