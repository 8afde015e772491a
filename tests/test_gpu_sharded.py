"""GPU: the sharded encrypted search (BASELINE configs[3]) on a
real device, rehearsed with 2 torch.distributed ranks sharing GPU 0 over gloo.

The 8-GPU RCCL run is the driver's; what this covers is everything below the
backend: every rank builds the same model and keys, takes its contiguous
document range of the store (index.json order, encrypted_storage.py:136-141),
runs the fused encrypted compare + encrypted threshold + local top-k in HIP
(`fhe_compare_batch`, `fhe_topk`), and the ranks meet in ONE all-gather of k
(acc, index) pairs (fheicp.search.sharded_topk). Every rank's result must be
the reference's sequential loop (batch_operations.py:268-284: float `>=`,
stable sort by score desc, `[:top_k]`) over the WHOLE store, restated by the
oracle (oracle/quant_ref.search)."""
import json
import multiprocessing as mp
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

from oracle import quant_ref as Q

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, store_dir, query, cases, q):
    for p in (str(REPO / "fhe-icp_amd"), str(REPO)):
        if p not in sys.path:
            sys.path.insert(0, p)
    try:
        import torch
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.cuda.set_device(0)               # both ranks share GPU 0
        torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
        from batch_operations import BatchConfig, BatchProcessor
        from encrypted_storage import EncryptedDocumentStore
        from fheicp import _lib
        cfg = BatchConfig(fhe="execute", input_dim=16, n_bits=6, seed=21, key_seed=22, search_chunk=128,
                          show_progress=False, key_manager_default=False)
        p = BatchProcessor(storage=EncryptedDocumentStore(store_dir), config=cfg)
        eng = p.fhe_model.model._fitted().engine
        eng.profile(True)
        res = [p.search_vector(np.asarray(query), k, t) for k, t in cases]
        torch.cuda.synchronize()
        eng.profile(False)
        brs = {g: eng.profile_read(f"blind_rotate_{g}")["items"] for g in ("main", "mid0", "mid", "mid2", "fast", "fast2")}
        from fheicp.params import sign_pbs_count
        brs["per_compare"] = sign_pbs_count(eng.params)
        q.put((rank, res, p.fhe_model.model.quant_params.to_dict(), brs, _lib.LIB_PATH and str(_lib.LIB_PATH)))
        torch.distributed.destroy_process_group()
    except BaseException as e:  # report instead of hanging the parent on q.get
        q.put((rank, repr(e), None, None, None))
        raise


def test_processor_sharded_encrypted_search_two_ranks(need_gpu, tmp_path, monkeypatch):
    """2 gloo ranks on GPU 0, BatchProcessor(fhe="execute").search_vector over
    a ragged 601-document store with duplicated documents on both sides of the
    rank boundary (index 300): each rank's returned list equals the oracle's
    restatement of batch_operations.py:268-284 over all 601 documents."""
    from encrypted_storage import EncryptedDocument, EncryptedDocumentStore
    monkeypatch.setattr(EncryptedDocument, "allowed_dims", (16, 128, 256))
    qv, docs = Q.make_corpus(16, 601, seed=91)
    docs[299] = docs[300]                       # tie straddling the boundary
    docs[12] = docs[450]
    docs[301] = docs[5]
    store = EncryptedDocumentStore(str(tmp_path))
    ids = [f"d{i:03d}" for i in range(len(docs))]
    store.save_many([EncryptedDocument(doc_id=ids[i], content_hash=f"{i:064x}", timestamp="2025-01-01T00:00:00",
                                       encrypted_embedding=docs[i], metadata={}) for i in range(len(docs))])
    cases = [(10, 0.5), (700, -100.0), (3, 100.0), (1, 0.0), (25, 0.3)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    ps = [ctx.Process(target=_rank_main, args=(r, world, port, str(tmp_path), qv.tolist(), cases, q))
          for r in range(world)]
    for p in ps:
        p.start()
    try:
        res = [q.get(timeout=300) for _ in ps]
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r, got, qd, _, _ in res:
        assert qd is not None, f"rank {r} failed: {got}"
    qp = Q.QuantizedLinearParams.from_json(res[0][2])
    for rank, got, qd, brs, lib in res:
        assert qd == res[0][2]
        # the encrypted path ran: this rank bootstrapped its own range only,
        # the sign extraction's bootstraps for each of its documents per case
        per_case = (301 if rank == 1 else 300)
        n_br = sum(v for g, v in brs.items() if g != "per_compare")
        assert n_br == brs["per_compare"] * per_case * len(cases), brs
        assert lib and lib.endswith("libfheicp.so")
        for (k, t), g in zip(cases, got):
            want = [(ids[i], s) for i, s in Q.search(qp, qv, docs, k, t)]
            assert g == want, (rank, k, t)


def test_bench_c4_two_ranks_gloo(need_gpu, tmp_path):
    """bench.py --workload c4 (configs[3]'s path at 4096 documents) under 2
    ranks sharing GPU 0: the timed sharded step, the per-rank parity against
    the clear restatement (all-reduced) and the merged top-10 against the
    global one."""
    env = dict(os.environ, FHEICP_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(REPO / "bench.py"),
           "--gpus", "2", "--workload", "c4", "--total-docs", "4096", "--steps", "1", "--warmup", "1"]
    r = subprocess.run(cmd, cwd=str(REPO), env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 2 and out["scaling"] == "strong"
    assert out["config"]["total_docs"] == 4096
    par = out["parity"]
    assert par["ranks"] == 2 and par["compares_checked"] == 4096
    assert par["acc_bit_exact"] and par["threshold_bit_exact"] and par["quant_params_equal"]
    assert out["topk_check"]["indices_equal"] and out["topk_check"]["scores_equal"]
    assert out["allgather_ms"] >= 0


def test_bench_gpus2_without_launcher(need_gpu):
    """`python bench.py --gpus 2` exactly as the driver invokes the N = 1 line
    (no torch.distributed.run, no WORLD_SIZE): bench.py must start the two
    ranks itself, and the line must be a 2-rank measurement with per-rank
    parity and the merged top-10 checked (gloo ranks sharing GPU 0)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(FHEICP_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--workload", "c4", "--total-docs", "4096",
           "--steps", "1", "--warmup", "1"]
    r = subprocess.run(cmd, cwd=str(REPO), env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "shard2"
    par = out["parity"]
    assert par["ranks"] == 2 and par["compares_checked"] == 4096
    assert par["acc_bit_exact"] and par["threshold_bit_exact"] and par["quant_params_equal"]
    assert out["topk_check"]["indices_equal"] and out["topk_check"]["scores_equal"]


def test_bench_one_rank_rccl(need_gpu):
    """The RCCL path on the one GPU of this box: bench.py under
    torch.distributed.run with one rank and the default backend ("nccl" =
    RCCL), so the process group, the barriers, the MAX/MIN/SUM all-reduces of
    the timing and parity flags and the top-k all-gather all execute on the
    device through RCCL (the 8-GPU run's code path, at world size 1)."""
    env = {k: v for k, v in os.environ.items() if k != "FHEICP_DIST_BACKEND"}
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(REPO / "bench.py"),
           "--gpus", "1", "--workload", "c4", "--total-docs", "4096", "--steps", "1", "--warmup", "1",
           "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=str(REPO), env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 1 and out["config"]["total_docs"] == 4096
    assert out["dist"]["backend"] == "nccl" and out["dist"]["rccl"] and out["dist"]["device"].startswith("cuda")
    par = out["parity"]
    assert par["ranks"] == 1 and par["compares_checked"] == 4096
    assert par["acc_bit_exact"] and par["threshold_bit_exact"] and par["quant_params_equal"]
    assert out["topk_check"]["indices_equal"] and out["topk_check"]["scores_equal"]
    assert out["allgather_ms"] > 0
    assert "local copy" in out["allgather_note"]   # world 1: not an xGMI number
    assert "RCCL top-k all-gather" in out["config"]["workload"]
