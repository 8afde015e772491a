"""Host-only checks of bench.py's launch contract (no GPU): --gpus must agree
with the launcher's WORLD_SIZE, and a direct `--gpus N` run starts N ranks
itself through torch.distributed.run (rendezvous on 127.0.0.1)."""
import os
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def test_world_size_mismatch_exits_nonzero():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "8", "--steps", "1"],
                       cwd=str(REPO), env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "--gpus 8 but WORLD_SIZE=2" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_rank_launch_cmd():
    sys.path.insert(0, str(REPO))
    import bench
    cmd = bench.rank_launch_cmd(4, ["--gpus", "4", "--steps", "3"])
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert int(cmd[cmd.index("--master-port") + 1]) > 0
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]
    assert cmd[-5] == str(REPO / "bench.py")


def test_packed_allgather_gloo_two_ranks(tmp_path):
    """The sharded top-k's single all-gather of packed [k, 2] pairs on a gloo
    world of 2 (the exchange bench.py and BatchProcessor use)."""
    code = r"""
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, sys.argv[1])
from fheicp.search import sharded_topk, host_topk
rank = int(os.environ["RANK"])
dist.init_process_group("gloo")
calls = []
orig = dist.all_gather
def counting(*a, **k):
    calls.append(a[1].shape)
    return orig(*a, **k)
dist.all_gather = counting
acc = torch.tensor([5, 9, 9, 1] if rank == 0 else [9, 7, 5, 9], dtype=torch.int64)
below = torch.zeros(4, dtype=torch.int64)
oa, oi = sharded_topk(acc, below, 3, rank * 4, host_topk, 2)
assert len(calls) == 1 and tuple(calls[0]) == (3, 2), calls
assert oa.tolist() == [9, 9, 9] and oi.tolist() == [1, 2, 4], (oa, oi)
dist.destroy_process_group()
open(os.path.join(sys.argv[2], f"ok{rank}"), "w").close()
"""
    script = tmp_path / "ag.py"
    script.write_text(code)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(script),
           str(REPO / "fhe-icp_amd"), str(tmp_path)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert (tmp_path / "ok0").exists() and (tmp_path / "ok1").exists()


def _port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_leveled_ops_model():
    """bench.leveled_ops_per_pair (the k_encrypt_linear roofline's algorithmic
    work): one kN-word GLWE mask per chunk of N features (kN / 8 ChaCha20
    blocks), ceil(Dg / 8) noise blocks per chunk, D x kN u64 multiply-adds."""
    sys.path.insert(0, str(REPO))
    import bench
    from fheicp.params import params_for_bits
    p = params_for_bits(16)
    kN = p.k * p.N
    assert bench.leveled_ops_per_pair(p, 16) == bench.CHACHA_BLOCK_OPS * (kN // 8 + 2) + bench.U64_MAC_OPS * kN * 16
    # two chunks past N features (1100 = 1024 + 76): two masks, 128 + 10 noise blocks
    assert bench.leveled_ops_per_pair(p, 1100) == (bench.CHACHA_BLOCK_OPS * (2 * kN // 8 + 128 + 10)
                                                   + bench.U64_MAC_OPS * kN * 1100)


def test_leveled_mix_floor():
    """The mix-aware floor of k_encrypt_linear: blocks x (ChaCha20 at the
    measured add / xor / alignbit rates) + MACs x (mad_u64 + 2 mul_lo + add3),
    linear in the pairs; the plain ops model at the dual-issue peak is faster."""
    sys.path.insert(0, str(REPO))
    import bench
    from fheicp.params import params_for_bits
    p = params_for_bits(16)
    assert bench.leveled_blocks_per_pair(p, 16) == 258
    f1 = bench.leveled_mix_floor_s(p, 16, 1)
    assert abs(bench.leveled_mix_floor_s(p, 16, 1024) - 1024 * f1) < 1e-15
    assert f1 > bench.leveled_ops_per_pair(p, 16) / (bench.VALU_PEAK_TOPS * 1e12)


def test_one_rank_launcher_creates_the_group(tmp_path):
    """WORLD_SIZE=1 under a launcher: dist_setup joins a process group (gloo
    here, RCCL on the GPU box) and sharded_topk runs its all-gather, so a
    one-GPU launcher run exercises the N-rank code path."""
    code = r"""
import os, sys, torch
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2])
import bench
from fheicp.search import sharded_topk, host_topk
class A: pass
world, rank, local = bench.dist_setup(A())
assert (world, rank) == (1, 0) and bench.dist_on()
assert torch.distributed.get_backend() == "gloo"
calls = []
orig = torch.distributed.all_gather
torch.distributed.all_gather = lambda *a, **k: (calls.append(1), orig(*a, **k))[1]
oa, oi = sharded_topk(torch.tensor([3, 8, 8, 1]), None, 2, 10, host_topk, 1)
assert calls == [1] and oa.tolist() == [8, 8] and oi.tolist() == [11, 12], (calls, oa, oi)
# a world that is not the group's is refused, not silently replaced
try:
    sharded_topk(torch.tensor([3, 8]), None, 1, 0, host_topk, 2)
    raise SystemExit("world 2 in a 1-rank group was accepted")
except ValueError:
    pass
torch.distributed.destroy_process_group()
open(os.path.join(sys.argv[3], "ok"), "w").close()
"""
    script = tmp_path / "one.py"
    script.write_text(code)
    env = dict(os.environ, FHEICP_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(script),
           str(REPO / "fhe-icp_amd"), str(REPO), str(tmp_path)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert (tmp_path / "ok").exists()


def test_bare_single_rank_has_no_group():
    """Run bare at N = 1 (the driver's default line) no group exists and
    sharded_topk is the local top-k alone."""
    sys.path.insert(0, str(REPO))
    import torch
    from fheicp.search import sharded_topk, host_topk
    assert not torch.distributed.is_initialized()
    oa, oi = sharded_topk(torch.tensor([1, 5]), None, 1, 0, host_topk, 1)
    assert oa.tolist() == [5] and oi.tolist() == [1]


def test_pipe_split_matches_the_library_halves():
    """bench.pipe_split mirrors fheicp.hip sign_extract_batch's halves: the
    first a whole number of 1024-ciphertext waves nearest count / 2 (from 2048
    ciphertexts), so the isolated launches time the step's real sizes."""
    import bench
    assert bench.pipe_split(12500) == (6144, 6356)
    assert bench.pipe_split(10000) == (5120, 4880)
    assert bench.pipe_split(2048) == (1024, 1024)
    assert bench.pipe_split(2050) == (1024, 1026)
    assert bench.pipe_split(1000) == (500, 500)
    for n in (2048, 3000, 4095, 4096, 12500, 100000):
        c0, c1 = bench.pipe_split(n)
        assert c0 % 1024 == 0 and c0 + c1 == n and c1 >= 4 and abs(c0 - n / 2) <= 512


def test_pipe_min_override_is_clamped_like_the_library(monkeypatch):
    """FHEICP_PIPE_MIN below 8 is clamped to 8 in bench.py as in
    fheicp.hip sign_extract_batch, so pipelined() / pipe_split() describe
    the launches the library makes."""
    import importlib
    sys.path.insert(0, str(REPO))
    import bench
    monkeypatch.setenv("FHEICP_PIPE_MIN", "4")
    b = importlib.reload(bench)
    try:
        assert b.PIPE_MIN == 8 and not b.pipelined(6) and b.pipelined(8)
    finally:
        monkeypatch.delenv("FHEICP_PIPE_MIN")
        importlib.reload(bench)
