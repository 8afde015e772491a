#!/usr/bin/env python3
"""Encrypted-compare throughput on MI355X (BASELINE.json metric).

Workload at N = 1 (BASELINE.json configs[1], the metric's config): one query
against 1024 documents, 16-dim features, n_bits = 6. At N > 1 (or with
--workload c4) the north-star scaling workload, configs[3]: a 100k-document
search, 16-dim, n_bits = 6, the corpus sharded over the ranks in contiguous
global index ranges (strong scaling: the total is fixed). One step = one pass
of the whole encrypted path over each rank's shard, all on the GPU:
    pair features + quantize -> packed GLWE encryption of the features fused
    with the leveled dot product (one GLWE mask per pair, k_encrypt_linear)
    -> decrypt the accumulator -> exact sign extraction of acc - T in 4-bit
    digits (fhe_sign_pbs_count key switches + bootstraps per pair: 7 at
    P = 16, on the multi-bit (15,2) and (23,1) rotations)
    -> decrypt the encrypted threshold bit -> local top-k
and, whenever a process group exists (any launcher run, N = 1 included), the
RCCL all-gather of the per-shard top-k (the only exchange step of the sharded
search) plus the merge.
Inputs (query, documents) are resident in HBM before the timed region.
value = compares processed by all ranks / (max over ranks of the time).

Launch: python bench.py [--gpus N --steps K --warmup W]. For N > 1 either
under torch.distributed.run (one process per GPU, RCCL = backend "nccl";
WORLD_SIZE must equal --gpus), or directly: the process then starts the N
ranks itself (launch_ranks) and relays rank 0's line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
for _p in (str(REPO / "fhe-icp_amd"), str(REPO)):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "encrypted compares/sec (PBS/sec), 16-dim, 1/2/4/8 GPU; bit-exact vs CPU"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md, HBM3E spec
F64_VALU_PEAK_TFLOPS = 78.6    # MI355X FP64 vector peak (AMD spec: 256 CUs x 128 FLOP/clk x 2.4 GHz)
PEAK_CLOCK_MHZ = 2400.0        # the clock F64_VALU_PEAK_TFLOPS is quoted at
# PMC measurement of this build's blind-rotation kernels (tools/pmc_bench.sh ->
# tools/br_pmc.py): executed f64 FLOPs and HBM bytes per launch, keyed on the
# sha256 of the libfheicp.so they were measured on
PMC_FILE = REPO / "profiles" / "br_pmc.json"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=("auto", "c2", "c4"), default="auto",
                    help="c2: configs[1], --docs per GPU (weak); c4: configs[3], --total-docs over all ranks "
                         "(strong); auto: c2 at N=1, c4 at N>1")
    ap.add_argument("--docs", type=int, default=1024, help="documents per GPU (c2 shard size)")
    ap.add_argument("--total-docs", type=int, default=100_000, help="documents over all ranks (c4)")
    ap.add_argument("--dim", type=int, default=16)
    ap.add_argument("--n-bits", type=int, default=6)
    ap.add_argument("--top-k", type=int, default=10)
    ap.add_argument("--min-similarity", type=float, default=0.5)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-compares", type=int, default=0,
                    help="oracle sample size (0: 64 compares scaled down by the sign plan's cost, 10-30 s)")
    ap.add_argument("--mode", choices=("compare", "corpus", "embed", "lut"), default="compare",
                    help="compare: the reference's path (configs[1]); corpus: search over a stored corpus of "
                         "seeded-LWE documents (SURVEY.md §8f-1); embed: the BERT encoder of the embedding "
                         "stage (SURVEY.md §8f-4); lut: the programmable (table) bootstrap, PBS/s (SURVEY.md "
                         "§8a row P, the north star's 'polynomial activation')")
    ap.add_argument("--lut-bits", type=int, default=4, help="--mode lut: input message bits of the table")
    ap.add_argument("--lut-msg-bits", type=int, default=16,
                    help="--mode lut: output width P (the parameter set params_for_bits(P))")
    ap.add_argument("--embed-batch", type=int, default=256, help="--mode embed: sequences per forward pass")
    ap.add_argument("--seq-len", type=int, default=100, help="--mode embed: tokens per sequence (max_length)")
    ap.add_argument("--embed-precision", choices=("f32", "bf16"), default="f32",
                    help="--mode embed: the encoder's arithmetic (f32: the reference's, on the f32 MFMA)")
    return ap.parse_args()


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_launch_cmd(gpus: int, argv: list[str]) -> list[str]:
    """The torch.distributed.run line that starts one rank per GPU on this
    node (the driver's own form, rendezvous on 127.0.0.1), forwarding argv."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
            str(Path(__file__).resolve())] + list(argv)


def launch_ranks(args, argv: list[str]) -> int | None:
    """--gpus N against the process layout, before anything touches the GPU.

    Under a launcher (WORLD_SIZE set) the world must be --gpus: a mismatch
    exits non-zero instead of measuring another GPU count. Invoked directly
    with --gpus N > 1, this process starts the N ranks itself as a child
    torch.distributed.run (no exec: it never initialises the GPU) and returns
    the child's exit code; rank 0's JSON line reaches stdout unchanged.
    None: this process is the (only) rank."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}", file=sys.stderr)
            return 2
        return None
    if args.gpus < 1:
        print(f"bench.py: --gpus {args.gpus}", file=sys.stderr)
        return 2
    if args.gpus == 1:
        return None
    import signal
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    child = subprocess.Popen(rank_launch_cmd(args.gpus, argv), env=env)
    # forward a termination to the launcher, which stops its ranks
    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, lambda s, _f: child.send_signal(s))
    return child.wait()


def dist_on() -> bool:
    """A process group exists: every collective of the run keys on this, not
    on world > 1, so a one-rank launcher run executes the RCCL path too."""
    return torch.distributed.is_available() and torch.distributed.is_initialized()


def dist_setup(args):
    """Under a launcher (WORLD_SIZE set, any size, 1 included) this joins the
    process group, RCCL (backend "nccl") bound to this rank's GPU unless
    FHEICP_DIST_BACKEND says otherwise; run bare at N = 1 it creates none."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if "WORLD_SIZE" in os.environ:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # one process per GPU; FHEICP_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs
        backend = os.environ.get("FHEICP_DIST_BACKEND", "nccl")
        local = local % max(torch.cuda.device_count(), 1)
        if torch.cuda.is_available():
            torch.cuda.set_device(local)
        if backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            torch.distributed.init_process_group(backend)
    return world, rank, local


def build_model(args):
    from fheicp.model import FheLinearModel
    from fheicp.datagen import training_pairs
    X, y = training_pairs(args.dim, 1000, seed=args.seed + 1)
    return FheLinearModel.fit(X, y, n_bits=args.n_bits)


def shard(args, rank, world=1):
    """(query, this rank's documents, global index of its first document).
    c2: every rank draws its own --docs documents (weak scaling); c4: one
    global corpus of --total-docs documents, rank r owns the contiguous range
    [r*T/N, (r+1)*T/N) (index.json insertion order, encrypted_storage.py:136-141)."""
    from fheicp.datagen import corpus
    if args.workload == "c4":
        q, docs = corpus(args.dim, args.total_docs, seed=args.seed + 100, query_seed=args.seed + 99)
        lo, hi = rank * args.total_docs // world, (rank + 1) * args.total_docs // world
        return q, docs[lo:hi], lo
    q, docs = corpus(args.dim, args.docs, seed=args.seed + 100 + rank, query_seed=args.seed + 99)
    return q, docs, rank * args.docs


def config_tag(args) -> str:
    """Which BASELINE.json config this run is (configs[1] is the metric's)."""
    if args.workload == "c4":
        return " (BASELINE configs[3])" if (args.total_docs, args.dim, args.n_bits) == (100_000, 16, 6) \
            else " (custom)"
    known = {(1024, 16, 6): "configs[1]", (10000, 32, 8): "configs[2] (one GPU)",
             (12500, 16, 6): "configs[3], one GPU's share of 100k docs", (1000, 768, 8): "configs[4]"}
    tag = known.get((args.docs, args.dim, args.n_bits))
    return f" (BASELINE {tag})" if tag else " (custom)"


def br_flops_per_ct(p, group: int = 1) -> float:
    """Analytic f64 FLOPs of one blind rotation (radix-2 FFT count, DESIGN.md
    §4.2); used only when no PMC measurement of this build exists. Group 2
    (multi-bit, §4.5): per pair of LWE coefficients the transforms of one
    step, three subsets' products and the (psi^(a e) - 1) factors."""
    M = p.N // 2
    logm = int(np.log2(M))
    fft = 5.0 * M * logm + 6.0 * M             # radix-2 complex FFT + twist
    nf, ni = (p.k + 1) * p.pbs_level, p.k + 1
    if group == 2:
        per_pair = nf * fft + ni * fft + 3 * 8.0 * nf * ni * M + p.pbs_level * 3 * ni * 9.0 * M
        return (p.n + 1) // 2 * per_pair
    pointwise = 8.0 * nf * ni * M
    return p.n * (nf * fft + ni * fft + pointwise)


def lib_sha256() -> str:
    import hashlib
    from fheicp import _lib
    return hashlib.sha256(Path(_lib.LIB_PATH).read_bytes()).hexdigest()


def load_pmc() -> dict:
    """Per-kernel PMC figures of THIS build, keyed "kernel@cts" ({} if the
    file was measured on another libfheicp.so)."""
    try:
        d = json.loads(PMC_FILE.read_text())
    except (OSError, ValueError):
        return {}
    return d.get("kernels", {}) if d.get("lib_sha256") == lib_sha256() else {}


def pmc_entry(pmc: dict, kernel: str, cts: int):
    """(entry at this batch size or None, any entry of this kernel or None)."""
    exact = pmc.get(f"{kernel}@{cts}")
    anyk = exact or next((v for k, v in pmc.items() if k.rsplit("@", 1)[0] == kernel), None)
    return exact, anyk


def read_br(eng) -> dict:
    """Blind-rotation HIP-event totals per gadget (fhe_profile_read) and the
    instantiation each launched (fhe_profile_kernel_name)."""
    out = {}
    for g in ("main", "mid0", "mid", "mid2", "fast", "fast2"):
        out[g] = eng.profile_read(f"blind_rotate_{g}")
        out[g]["kernel"] = eng.kernel_name(f"blind_rotate_{g}")
    return out


def _br_kernel(q, br, pmc, group: int = 1) -> dict:
    """One blind-rotation kernel (gadget q) from its own launches: HIP-event
    time per launch; f64 FLOPs executed per launch from the PMC pass of this
    build at this batch size (else the analytic count); algorithmic HBM bytes
    (the FFT-domain BSK once + LWE I/O) and the PMC-measured HBM bytes."""
    avg_ms = br["total_ms"] / max(br["launches"], 1)
    cts_per_launch = br["items"] / max(br["launches"], 1)
    ggsws = 3 * ((q.n + 1) // 2) if group == 2 else q.n
    bsk_bytes = ggsws * (q.k + 1) * q.pbs_level * (q.k + 1) * (q.N // 2) * 16
    io_bytes = cts_per_launch * ((q.n + 1) * 8 + (q.k * q.N + 1) * 8 * 5)
    alg_bytes = bsk_bytes + io_bytes
    m, anyk = pmc_entry(pmc, br["kernel"], int(round(cts_per_launch)))
    m = m or {}
    # executed f64 FLOPs: PMC of this build (per padded ciphertext, so any
    # batch of the same kernel); the analytic radix-2 count only when this
    # kernel was never measured on this build (it over-counts by 14-20%)
    padded = (int(round(cts_per_launch)) + 3) // 4 * 4
    measured = anyk is not None and "f64_flops_per_ct" in anyk
    flops = float(anyk["f64_flops_per_ct"]) * padded if measured else br_flops_per_ct(q, group) * cts_per_launch
    secs = avg_ms * 1e-3
    return {
        "kernel": br["kernel"], "gadget": [q.pbs_base_log, q.pbs_level], "group": group,
        "avg_launch_ms": round(avg_ms, 4), "launches": br["launches"], "cts_per_launch": cts_per_launch,
        "total_ms": round(br["total_ms"], 3),
        "f64_flops_per_launch": flops, "flops_source": "pmc" if measured else "analytic",
        "achieved_tflops_f64": flops / secs / 1e12 if br["launches"] else 0.0,
        "alg_bytes_per_launch": int(alg_bytes),
        "achieved_gbs": alg_bytes / secs / 1e9 if br["launches"] else 0.0,
        # HBM bytes do not scale with the batch (each XCD's L2 streams the key once): exact batch only
        "hbm_bytes_per_launch": float(m["hbm_bytes_per_launch"]) if "hbm_bytes_per_launch" in m else None,
        # the clock the kernel held in the PMC pass (GRBM_GUI_ACTIVE / 8 XCDs /
        # dispatch time): the f64-heavy kernels run below the 2.4 GHz the peak
        # is quoted at (power), so frac_at_clock prices them at their own clock
        "clock_mhz": (anyk or {}).get("clock_mhz"),
        "pmc_avg_launch_ms": m.get("avg_launch_ms"),
        "pmc_command": (anyk or {}).get("command"),
    }


# fhe_compare_batch splits batches of >= 2048 ciphertexts into two halves on
# two streams (fheicp.hip PIPE_MIN, FHEICP_PIPE=0 turns it off)
# (the library clamps an override to >= 8: sign_extract_batch)
PIPE_MIN = max(8, int(os.environ.get("FHEICP_PIPE_MIN", "2048")))


def pipelined(batch: int) -> bool:
    return batch >= PIPE_MIN and os.environ.get("FHEICP_PIPE", "1") != "0"


GADGET_ID = {"main": 0, "fast": 1, "fast2": 2, "mid": 3, "mid2": 4, "mid0": 5}


def pipe_split(count: int):
    """The two halves fhe_compare_batch's pipelined sign extraction launches
    (fheicp.hip sign_extract_batch: the first a whole number of
    1024-ciphertext waves nearest count / 2)."""
    if count < 2048:
        c0 = ((count // 2) + 3) & ~3
    else:
        c0 = min(max(1024, 1024 * ((count + 1024) // 2048)), count - 4)
    return c0, count - c0


def isolated_br(eng, brs, batch: int, reps: int = 3) -> dict:
    """Per-kernel launch times without the pipelined step's overlap: every
    blind-rotation kernel the step launched, run alone (fhe_pbs_gadget_batch,
    one stream) at the step's two half-batch sizes (pipe_split) on fresh
    key-switched inputs, HIP events around each launch (after the timed
    region); the totals cover both halves, so avg_launch_ms and
    cts_per_launch are those of the step's launches."""
    out = {}
    halves = pipe_split(batch)
    for g, b in brs.items():
        if not b["launches"]:
            continue
        tot = None
        for cts in halves:
            v = np.where(np.arange(cts) % 2 == 0, 1, -1).astype(np.int64) << 10
            small = eng.keyswitch(eng.encrypt(v, seed=99), 0, 0)
            eng.pbs_gadget(small, GADGET_ID[g], 1 << 61)        # warm-up
            torch.cuda.synchronize()
            eng.profile(True)
            for _ in range(reps):
                eng.pbs_gadget(small, GADGET_ID[g], 1 << 61)
            torch.cuda.synchronize()
            eng.profile(False)
            r = eng.profile_read(f"blind_rotate_{g}")
            r["kernel"] = eng.kernel_name(f"blind_rotate_{g}")
            assert r["kernel"] == b["kernel"], (r["kernel"], b["kernel"])
            if tot is None:
                tot = r
            else:
                for key in ("launches", "items", "total_ms"):
                    tot[key] += r[key]
            del small
        tot["halves"] = list(halves)
        out[g] = tot
    return out


def roofline(p, brs, batch: int = 0, iso: dict | None = None) -> dict:
    """Roofline of the dominant blind-rotation (external-product) kernel.

    The kernel is f64-VALU bound (the FFT-domain BSK stream is
    L2/Infinity-cache resident and its HBM rate is ~0.3% of 8 TB/s), so the
    roof is the f64 vector peak: achieved = f64 FLOPs executed per launch
    (rocprofv3 SQ_INSTS_VALU_{FMA,ADD,MUL}_F64 of this exact build, x64 lanes,
    FMA x2) / the HIP-event launch time on the kernel's stream. The HBM view
    (algorithmic bytes / time against 8 TB/s, and the PMC-measured bytes as
    `traffic`) stays beside it. With per-round gadgets up to
    six gadgets run; the kernel with the largest total time is reported, all
    are listed under `kernels`."""
    from dataclasses import replace
    from fheicp.params import gadget_level, gadget_of
    qs = {}
    for g, gid in (("main", 0), ("mid0", 5), ("mid", 3), ("mid2", 4), ("fast", 1), ("fast2", 2)):
        if gid == 0 or gadget_level(p, gid):
            bl, lv, grp = gadget_of(p, gid)
            qs[g] = (replace(p, pbs_base_log=bl, pbs_level=lv), grp)
    pmc = load_pmc()
    ks = {g: _br_kernel(q, brs[g], pmc, grp) for g, (q, grp) in qs.items() if brs[g]["launches"]}
    dom = max(ks, key=lambda g: ks[g]["total_ms"])
    if iso:
        # pipelined step: the launch times come from the isolated launches,
        # the in-step (overlapped) ones stay beside them
        for g in ks:
            step_ms = ks[g]["avg_launch_ms"]
            ks[g] = _br_kernel(qs[g][0], iso[g], pmc, qs[g][1])
            ks[g]["in_step_avg_launch_ms"] = step_ms
            ks[g]["total_ms"] = round(step_ms * brs[g]["launches"], 3)
            ks[g]["launches"] = brs[g]["launches"]
    k = ks[dom]
    tf = k["achieved_tflops_f64"]
    clk = k.get("clock_mhz")
    return {
        "kernel": k["kernel"],
        "bound": "f64-valu",
        "achieved": round(tf, 3),
        "peak": F64_VALU_PEAK_TFLOPS,
        "unit": "TFLOP/s",
        "frac": round(tf / F64_VALU_PEAK_TFLOPS, 4),
        "clock_mhz": clk,
        "frac_at_clock": round(tf / (F64_VALU_PEAK_TFLOPS * clk / PEAK_CLOCK_MHZ), 4) if clk else None,
        "traffic": k["hbm_bytes_per_launch"],
        "flops_per_launch": k["f64_flops_per_launch"],
        # a pipelined step runs two half-batch launches at once, so its
        # per-launch times include the other half's kernel: `achieved` then
        # uses the same kernel's isolated launches at the same batch
        "overlapped_launches": pipelined(batch) and not iso,
        "time_source": ("isolated launches at the step's two half-batch sizes after the timed region "
                        "(pipelined step)"
                        if iso else "HIP events on the step's launches"),
        "flops_source": k["flops_source"],
        "avg_launch_ms": k["avg_launch_ms"],
        "launches": k["launches"],
        "cts_per_launch": k["cts_per_launch"],
        "hbm": {"alg_bytes_per_launch": k["alg_bytes_per_launch"], "achieved_gbs": round(k["achieved_gbs"], 2),
                "peak_gbs": HBM_PEAK_GBS, "frac": round(k["achieved_gbs"] / HBM_PEAK_GBS, 5),
                "traffic_bytes_per_launch": k["hbm_bytes_per_launch"]},
        "pmc": {"file": str(PMC_FILE.relative_to(REPO)), "matches_this_build": bool(pmc),
                "recipe": "f64 FLOPs = 64 x (2 FMA_F64 + ADD_F64 + MUL_F64) wave-instructions; HBM bytes = "
                          "(2 x FETCH_SIZE + WRITE_SIZE) x 1024 (gfx950 FETCH_SIZE half-count), separate --pmc "
                          "passes over bench.py --steps 1"},
        "kernels": {g: {kk: (round(v, 3) if isinstance(v, float) else v) for kk, v in kv.items()}
                    for g, kv in ks.items()},
    }


def main():
    args = parse()
    code = launch_ranks(args, sys.argv[1:])
    if code is not None:
        sys.exit(code)
    world, rank, local = dist_setup(args)
    if args.workload == "auto":
        args.workload = "c4" if world > 1 else "c2"
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    from fheicp import _lib
    _lib.lib()  # loud failure if the HIP library is missing
    if args.mode == "corpus":
        return corpus_main(args, world, rank, local, dev)
    if args.mode == "embed":
        return embed_main(args, world, rank, local, dev)
    if args.mode == "lut":
        return lut_main(args, world, rank, local, dev)

    model = build_model(args)
    model.compile(key_seed=args.seed, device=local)
    eng = model.engine
    p = eng.params
    P = model.msg_bits
    from fheicp.params import sign_pbs_count
    n_pbs = sign_pbs_count(p)
    from fheicp.model import threshold_int
    from fheicp.search import sharded_topk
    T = threshold_int(model.qparams, args.min_similarity)

    q_np, docs_np, base_idx = shard(args, rank, world)
    q_dev = torch.from_numpy(q_np).to(dev)
    d_dev = torch.from_numpy(docs_np).to(dev)
    B = docs_np.shape[0]

    def step():
        qx = model.quantize_dev(d_dev, q_dev)
        acc, below = model.encrypted_acc(qx, T)
        oa, oi = sharded_topk(acc, below, args.top_k, base_idx, eng.topk, world)
        return acc, below, oa, oi

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    eng.profile(True)
    if dist_on():
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        acc, below, oa, oi = step()
    torch.cuda.synchronize()
    if dist_on():
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    eng.profile(False)
    br = read_br(eng)
    ks = eng.profile_read("keyswitch")

    if dist_on():
        on_dev = torch.distributed.get_backend() == "nccl"
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if on_dev else "cpu")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())

    compares = (args.total_docs if args.workload == "c4" else world * B) * args.steps
    value = compares / elapsed
    ms_step = elapsed / args.steps * 1e3

    roof = roofline(p, br, B, isolated_br(eng, br, B) if pipelined(B) else None)
    # every rank checks its own shard against the clear restatement of the
    # reference path; the flags meet in one all-reduce (MIN)
    par = shard_parity(args, model, q_np, docs_np, acc, below, T)
    if dist_on():
        flags = torch.tensor([int(par["acc_bit_exact"]), int(par["threshold_bit_exact"]),
                              int(par["quant_params_equal"]), par["compares_checked"]], dtype=torch.int64)
        on_dev = torch.distributed.get_backend() == "nccl"
        mins, tot = flags[:3].to(dev if on_dev else "cpu"), flags[3:].to(dev if on_dev else "cpu")
        torch.distributed.all_reduce(mins, op=torch.distributed.ReduceOp.MIN)
        torch.distributed.all_reduce(tot, op=torch.distributed.ReduceOp.SUM)
        mins, tot = mins.cpu().tolist(), int(tot.item())
        par = {"compares_checked": tot, "ranks": world, "acc_bit_exact": bool(mins[0]),
               "threshold_bit_exact": bool(mins[1]), "quant_params_equal": bool(mins[2])}
        allgather_ms = time_allgather(args.top_k, dev, on_dev)

    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "compares/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "strong" if args.workload == "c4" else "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic",
        "config": {
            "workload": (f"search 1 query over {args.total_docs} encrypted docs sharded over {world} GPU(s)"
                         if args.workload == "c4" else f"batch compare 1 query x {B} encrypted docs per GPU")
                        + f", {args.dim}-dim, n_bits={args.n_bits}"
                        f"{config_tag(args)} + encrypted threshold (min_similarity {args.min_similarity}) "
                        f"+ top-{args.top_k}" + (" + RCCL top-k all-gather" if dist_on() else ""),
            "docs_per_gpu": B, "total_docs": args.total_docs if args.workload == "c4" else world * B,
            "dim": args.dim, "n_bits": args.n_bits, "msg_bits_P": P,
            "pbs_per_compare": n_pbs, "keyswitch_per_compare": n_pbs,
            "params": p.as_dict(), "parallelism": f"shard{world}",
        },
        "pbs_per_sec": round(value * n_pbs, 1),
        "roofline": roof,
        "keyswitch_ms_total": round(ks["total_ms"], 3),
    }

    out["parity"] = par
    out["leveled_score"] = leveled_score(args, model, q_dev, d_dev, acc)
    if dist_on():
        out["allgather_ms"] = round(allgather_ms, 4)
        out["allgather_note"] = (
            "one all-gather of k (acc, index) pairs per rank, timed after the timed region; "
            + ("at world size 1 it is a local copy on the device, not an xGMI transfer" if world == 1 else
               f"{world} ranks' {args.top_k} x 16 B over "
               + ("RCCL (xGMI between GPUs)" if torch.distributed.get_backend() == "nccl" else
                  f"{torch.distributed.get_backend()} (host copies)")))
        out["dist"] = dist_info(dev)
    if world == 1:
        out["pcie_inclusive"] = pcie_inclusive(args, model, q_dev, docs_np, T, dev)
    if rank == 0:
        out["topk_check"] = topk_check(args, model, world, oa, oi)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_leg(args, model, q_np, docs_np, par)

    share_note(out, world)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist_on():
        torch.distributed.destroy_process_group()


def dist_info(dev) -> dict:
    """What ran the collectives: the backend and, for RCCL, the device it is
    bound to."""
    b = torch.distributed.get_backend()
    return {"backend": b, "rccl": b == "nccl", "world_size": torch.distributed.get_world_size(),
            "device": str(dev) if b == "nccl" else "cpu (host copies)"}


def share_note(out: dict, world: int) -> None:
    """Ranks sharing GPUs (a gloo rehearsal of N ranks on fewer cards): the
    per-launch kernel times include the other ranks' kernels, so the roofline
    is not a per-GPU figure; the line says so and carries it only as raw."""
    ngpu = torch.cuda.device_count()
    if world > ngpu:
        note = f"{world} ranks share {ngpu} GPU(s): kernel launch times overlap other ranks' kernels"
        out["config"]["gpu_sharing"] = note
        raw = out.pop("roofline", None)
        out["roofline"] = {"per_gpu": False, "note": note + "; the fraction below is not a per-GPU roofline",
                           "shared_raw": raw}


VALU_PEAK_TOPS = 78.6   # 32-bit VALU lane-ops/s: 256 CUs x 4 SIMD-32 x 32 lanes x 2.4 GHz (MI355X_MICROARCH.md)
CHACHA_BLOCK_OPS = 976  # one ChaCha20 block: 80 quarter rounds x 12 (add, xor, alignbit) + 16 final adds
U64_MAC_OPS = 4         # acc += w * a mod 2^64, small signed w: v_mad_u64_u32 + 2 v_mul_lo_u32 + v_add3_u32


# Issue rates of k_encrypt_linear's work at its occupancy (4 waves per SIMD),
# T lane-ops/s chip-wide, measured by tools/valu_probe.hip
# (profiles/r04_valu_probe.txt): VOP2 add/xor dual-issue, the VOP3 ops
# (v_alignbit_b32, v_mul_lo_u32, v_add3_u32, v_mad_u64_u32) do not; the
# product's own ChaCha20 block, one per lane, runs at 37.9 (976 ops each).
VALU_RATES_4W = {"add": 57.36, "xor": 58.57, "alignbit": 36.47, "mad_u64": 31.63, "mul_lo": 34.87, "add3": 35.46,
                 "chacha_block": 37.91}


def leveled_blocks_per_pair(p, D: int) -> int:
    G = -(-D // p.N)
    return G * (p.k * p.N // 8) + sum(-(-min(D - g * p.N, p.N) // 8) for g in range(G))


def leveled_mix_floor_s(p, D: int, B: int) -> float:
    """Seconds a launch of B pairs needs at the measured rates of its ops
    model: ChaCha20 blocks (336 v_add_u32, 320 v_xor_b32, 320 v_alignbit_b32)
    at the probe's rate for the real block, one per lane; a u64 MAC (one
    v_mad_u64_u32, two v_mul_lo_u32, one v_add3_u32) at each instruction's."""
    r = {k: v * 1e12 for k, v in VALU_RATES_4W.items()}
    chacha = CHACHA_BLOCK_OPS / r["chacha_block"]
    mac = 1 / r["mad_u64"] + 2 / r["mul_lo"] + 1 / r["add3"]
    return B * (leveled_blocks_per_pair(p, D) * chacha + p.k * p.N * D * mac)


def leveled_ops_per_pair(p, D: int) -> int:
    """Algorithmic 32-bit integer ops of one pair in k_encrypt_linear (packed
    features): the GLWE masks (kN / 8 ChaCha20 blocks per
    chunk), the features' noise words (ceil(Dg / 8) blocks per chunk) and the
    extraction's D x kN u64 multiply-adds."""
    return CHACHA_BLOCK_OPS * leveled_blocks_per_pair(p, D) + U64_MAC_OPS * p.k * p.N * D


def leveled_score(args, model, q_dev, d_dev, acc_compare) -> dict:
    """The reference's own encrypted predict (fhe_similarity.py:142-160):
    the leveled circuit only (encrypt + dot -> decrypt; fhe_score_batch, no
    key switch or bootstrap) over the same documents, inputs in HBM. Its
    accumulators must equal the compare path's (checked against the clear
    restatement in `parity`). Reported beside the headline, which adds the
    bootstrapped threshold bit. Roofline of its dominant kernel,
    k_encrypt_linear (the fused packed-GLWE encryption + dot product):
    integer-VALU bound (ChaCha20 mask generation + u64 multiply-adds; its HBM
    traffic is the 8 (kN + 1) output bytes per pair), algorithmic ops per
    launch over the HIP-event launch time against the 32-bit VALU peak."""
    eng = model.engine
    acc = model.encrypted_score(model.quantize_dev(d_dev, q_dev))
    torch.cuda.synchronize()
    reps = max(args.steps, 3)
    eng.profile(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        acc = model.encrypted_score(model.quantize_dev(d_dev, q_dev))
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    eng.profile(False)
    k = eng.profile_read("encrypt_linear")
    B = acc.shape[0]
    p = eng.params
    ops = leveled_ops_per_pair(p, args.dim) * B
    avg_s = k["total_ms"] / max(k["launches"], 1) * 1e-3
    tops = ops / avg_s / 1e12 if k["launches"] else 0.0
    out_bytes = 8 * (p.k * p.N + 1) * B
    # executed VALU instructions of this build (PMC, tools/pmc_bench.sh), x 64 lanes
    pm = load_pmc().get(f"k_encrypt_linear@{B}", {})
    pmc_ops = 64.0 * pm["valu_insts_per_launch"] if "valu_insts_per_launch" in pm else None
    return {"value": round(B * reps / el, 1), "unit": "scores/s", "ms_per_batch": round(el / reps * 1e3, 4),
            "acc_equal_to_compare": bool(torch.equal(acc, acc_compare)),
            "roofline": {"kernel": eng.kernel_name("encrypt_linear"), "bound": "valu-int",
                         "achieved": round(tops, 3), "peak": VALU_PEAK_TOPS, "unit": "Tops/s (32-bit lane ops)",
                         "frac": round(tops / VALU_PEAK_TOPS, 4), "avg_launch_ms": round(avg_s * 1e3, 5),
                         "launches": k["launches"], "pairs_per_launch": B,
                         "ops_per_pair": leveled_ops_per_pair(p, args.dim),
                         "ops_model": f"{CHACHA_BLOCK_OPS} per ChaCha20 block + {U64_MAC_OPS} per u64 MAC",
                         "valu_mix_floor_ms": round(leveled_mix_floor_s(p, args.dim, B) * 1e3, 5),
                         "mix_frac": round(leveled_mix_floor_s(p, args.dim, B) / avg_s, 4) if k["launches"] else 0.0,
                         "mix_rates": "tools/valu_probe.hip at 4 waves/SIMD (profiles/r04_valu_probe.txt)",
                         "pmc_valu_lane_ops_per_launch": pmc_ops,
                         "pmc_executed_frac": round(pmc_ops / avg_s / 1e12 / VALU_PEAK_TOPS, 4)
                         if pmc_ops and k["launches"] else None,
                         "hbm": {"bytes_per_launch": out_bytes,
                                 "achieved_gbs": round(out_bytes / avg_s / 1e9, 1) if k["launches"] else 0.0,
                                 "peak_gbs": HBM_PEAK_GBS}}}


def pcie_inclusive(args, model, q_dev, docs_np, T, dev) -> dict:
    """The same steps with the document embeddings handed over in (pinned)
    host memory and the accumulators and threshold bits copied back: the
    rate a caller with host buffers sees (never `value`, whose inputs are
    resident in HBM)."""
    d_host = torch.from_numpy(docs_np).pin_memory()
    B = docs_np.shape[0]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        d_in = d_host.to(dev, non_blocking=True)
        qx = model.quantize_dev(d_in, q_dev)
        acc, below = model.encrypted_acc(qx, T)
        acc.cpu(), below.cpu()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return {"value": round(B * args.steps / el, 2), "unit": "compares/s", "ms_per_step": round(el / args.steps * 1e3, 3),
            "h2d_bytes_per_step": int(d_host.numel() * d_host.element_size()), "d2h_bytes_per_step": 16 * B}


def topk_check(args, model, world, oa, oi):
    """The merged encrypted top-k of the last step (identical on every rank)
    against the global top-k of the product's clear quantized path over all
    ranks' shards: batch_operations.py:278-284 semantics (score >= t, stable
    sort by score desc, global document index breaking ties)."""
    scores = []
    for r in range(world):
        q, docs, _ = shard(args, r, world)
        scores.append(model.predict_clear(q[None, :] * docs))
    sc = np.concatenate(scores)
    keep = [(i, float(sc[i])) for i in range(len(sc)) if sc[i] >= args.min_similarity]
    keep.sort(key=lambda x: x[1], reverse=True)
    ref_idx = [i for i, _ in keep[:args.top_k]]
    got = [int(i) for i in oi.cpu().tolist() if i >= 0]
    s = np.float64(model.qparams.out_scale)
    got_scores = [float(s * np.float64(a)) for a, i in zip(oa.cpu().tolist(), oi.cpu().tolist()) if i >= 0]
    return {"docs": int(len(sc)), "k": args.top_k, "indices_equal": got == ref_idx,
            "scores_equal": got_scores == [sc_ for _, sc_ in keep[:args.top_k]]}


def cpu_sample(args, p) -> int:
    """Compares timed on the CPU oracle: --cpu-compares, or 64 at the
    headline's plan cost (3.9 relative bootstraps, about 12 s on 16 host
    threads) scaled down to the configuration's plan, at least 8."""
    if args.cpu_compares:
        return args.cpu_compares
    from fheicp.params import plan_cost
    return int(max(8, min(64, round(64 * 3.9 / max(plan_cost(p), 1e-9)))))


def shard_parity(args, model, q_np, docs_np, acc_dev, below_dev, T) -> dict:
    """The last timed step's accumulators and threshold bits of this rank's
    shard against the clear restatement of the reference path (the oracle's
    fit + quantize + accumulate, fhe_similarity.py:88-94, :167;
    batch_operations.py:226, :278)."""
    from oracle import quant_ref as Q
    X, y = __import__("fheicp.datagen", fromlist=["x"]).training_pairs(args.dim, 1000, seed=args.seed + 1)
    oq = Q.fit_quantized_linear(X, y, args.n_bits)
    acc_ref = Q.accumulate(oq, Q.quantize_input(oq, Q.pair_features(q_np, docs_np)))
    scores_ref = Q.dequantize(oq, acc_ref)
    return {
        "compares_checked": int(len(acc_ref)),
        "acc_bit_exact": bool(np.array_equal(acc_dev.cpu().numpy(), acc_ref)),
        "threshold_bit_exact": bool(np.array_equal(below_dev.cpu().numpy(),
                                                   (scores_ref < args.min_similarity).astype(np.int64))),
        "quant_params_equal": oq.to_json() == model.qparams.to_dict(),
    }


def time_allgather(k, dev, on_dev, iters=20) -> float:
    """Mean time of the search's one exchange step (one all-gather of k
    (acc, index) pairs per rank packed as [k, 2] int64, fheicp.search.sharded_topk), after the timed
    region so it does not perturb it."""
    a = torch.zeros(k, 2, dtype=torch.int64, device=dev if on_dev else "cpu")
    world = torch.distributed.get_world_size()
    outs = [torch.empty_like(a) for _ in range(world)]
    torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        torch.distributed.all_gather(outs, a)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def cpu_leg(args, model, q_np, docs_np, parity):
    """The oracle, timed on the host cores (bounded sample); adds its own
    agreement with the clear restatement to `parity`."""
    from oracle import quant_ref as Q
    from oracle import tfhe_ref as R
    X, y = __import__("fheicp.datagen", fromlist=["x"]).training_pairs(args.dim, 1000, seed=args.seed + 1)
    oq = Q.fit_quantized_linear(X, y, args.n_bits)
    Xp = Q.pair_features(q_np, docs_np)
    acc_ref = Q.accumulate(oq, Q.quantize_input(oq, Xp))
    T = Q.threshold_int(oq, args.min_similarity, *Q.acc_bounds(oq))
    # Oracle TFHE on C compares, the whole encrypted path: encrypt + linear +
    # decrypt + the digit sign extraction (all its KS + PBS) + decrypt.
    p = model.engine.params.as_dict()
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    C = cpu_sample(args, model.engine.params)
    ref = R.RefTFHE(p, args.seed)
    qx = Q.quantize_input(oq, Xp[:C])
    t0 = time.perf_counter()
    glwe = ref.encrypt_packed(qx, seed=5)          # packed features, as fhe_encrypt_linear_batch
    lin = ref.linear_packed(glwe, args.dim, oq.q_w, oq.const_term - T)
    v = ref.decrypt_ints(lin)
    bits = ref.decrypt_bits(ref.sign_extract(lin))
    t_total = time.perf_counter() - t0
    parity["cpu_oracle_acc_matches"] = bool(np.array_equal(v + T, acc_ref[:C]))
    parity["cpu_oracle_threshold_matches"] = bool(np.array_equal(bits, (acc_ref[:C] < T).astype(np.int64)))
    n_pbs = R.sign_pbs_count(p)
    base = {
        "value": round(C / t_total, 4),
        "unit": "compares/s",
        "cores": cores,
        "kind": "port",
        "sample": f"{C} compares of the same workload, the whole encrypted path on the exact C oracle (Karatsuba "
                  f"Z_2^64 TFHE, OpenMP {cores} threads): packed GLWE encrypt + linear + decrypt + {n_pbs} KS+PBS "
                  f"sign extraction + decrypt",
        "seconds": round(t_total, 2),
    }
    # the reference's shipped CPU path (Concrete predict fhe="disable": clear
    # quantized inference), numpy, single process
    t0 = time.perf_counter()
    reps = 200
    for _ in range(reps):
        Q.predict(oq, Xp)
    t_clear = (time.perf_counter() - t0) / reps
    base["clear_path_compares_per_s"] = round(len(Xp) / t_clear, 1)
    return base


def lut_main(args, world, rank, local, dev):
    """--mode lut: the programmable bootstrap with an arbitrary table
    (fhe_pbs_table_batch), the PBS a requantisation or a polynomial activation
    of the north star would run. --docs ciphertexts of random lut_bits-bit
    messages (one padding bit) are resident in HBM; one step = key switch +
    table bootstrap of all of them into P-bit outputs (a random signed
    table). The default gadget is the set's most precise multi-bit one, the
    sign extraction's kernel family (P = 16: (15,2), k_blind_rotate_mb<2, 0,
    15, BrTvLut>). Every output is decrypted against lut[m]; four phases
    against the oracle's ref_pbs_table_gadget on the same keys; the sign
    path's kernel on the same gadget and inputs is timed beside it."""
    from dataclasses import replace
    from fheicp.engine import Engine, u64
    from fheicp.params import gadget_of, params_for_bits
    P, lb, B = args.lut_msg_bits, args.lut_bits, args.docs
    p = params_for_bits(P)
    eng = Engine(p, local)
    eng.keygen(args.seed)
    gad = eng.table_gadget()
    rng = np.random.default_rng(args.seed + 3)
    M = 1 << lb
    lut = rng.integers(-(2 ** (P - 1)), 2 ** (P - 1), M)
    m = rng.integers(0, M, B)
    eng.set_msg_bits(lb + 1)                 # the input encoding: padding bit + lut_bits
    ct = eng.encrypt(m, seed=args.seed + 4)
    eng.set_msg_bits(P)
    lut_d = eng.to_dev(lut)
    small = eng.keyswitch(ct, 0, 0)

    def step():
        sm = eng.keyswitch(ct, 0, 0)
        return eng.pbs_table(sm, lut_d, lb)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    eng.profile(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    secs = time.perf_counter() - t0
    eng.profile(False)
    bucket = {0: "blind_rotate_main", 1: "blind_rotate_fast", 2: "blind_rotate_fast2", 3: "blind_rotate_mid",
              4: "blind_rotate_mid2", 5: "blind_rotate_mid0"}[gad]
    br = eng.profile_read(bucket)
    br["kernel"] = eng.kernel_name(bucket)
    ks = eng.profile_read("keyswitch")
    bl, lv, grp = gadget_of(p, gad)
    q = replace(p, pbs_base_log=bl, pbs_level=lv)
    k = _br_kernel(q, br, load_pmc(), grp)
    dec = eng.decrypt(out).cpu().numpy()
    exact = bool(np.array_equal(dec, lut[m]))
    # the sign extraction's kernel on the same gadget and inputs (constant
    # test vector, fhe_pbs_gadget_batch), the per-bootstrap yardstick
    for _ in range(2):
        eng.pbs_gadget(small, gad, 1 << 62)
    torch.cuda.synchronize()
    eng.profile(True)
    for _ in range(args.steps):
        eng.pbs_gadget(small, gad, 1 << 62)
    torch.cuda.synchronize()
    eng.profile(False)
    sg = eng.profile_read(bucket)
    sign_ms = sg["total_ms"] / max(sg["launches"], 1)
    sign_kernel = eng.kernel_name(bucket)
    oracle = {}
    if not args.no_cpu_baseline:
        from oracle import tfhe_ref as R
        R.build()
        ref = R.RefTFHE(p.as_dict(), args.seed)
        sm = u64(small)[:4]
        o_ref = ref.pbs_table(sm, lut, lb, gadget=gad)
        d = (u64(eng.phase(out[:4].contiguous())) - ref.phase(o_ref)).view(np.int64)
        oracle = {"compares": 4, "decrypt_equal": bool(np.array_equal(ref.decrypt_ints(o_ref), lut[m[:4]])),
                  "max_phase_diff_log2": round(float(np.log2(max(np.abs(d).max(), 1))), 2)}
        nthr = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
        cnt = 8
        sm8 = u64(small)[:cnt]
        t1 = time.perf_counter()
        ref.pbs_table(sm8, lut, lb, gadget=gad)
        cpu_s = time.perf_counter() - t1
        oracle["cpu_baseline"] = {"value": round(cnt / cpu_s, 3), "unit": "PBS/s", "cores": nthr, "kind": "port",
                                  "sample": f"{cnt} table bootstraps (ref_pbs_table_gadget, exact integer "
                                            f"restatement, OpenMP over the host cores)"}
    value = B * args.steps / secs
    tf = k["achieved_tflops_f64"]
    line = {
        "metric": "programmable bootstraps/sec (table PBS, key switch + blind rotation), 1 GPU",
        "value": round(value, 1), "unit": "PBS/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(secs / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u64", "data": "synthetic",
        "config": {"workload": f"table bootstrap of {B} ciphertexts: {lb}-bit inputs -> {P}-bit outputs "
                               f"(random signed table), params_for_bits({P}), gadget {gad} ({bl},{lv}) "
                               f"{'multi-bit' if grp == 2 else 'classic'}",
                   "ciphertexts": B, "lut_bits": lb, "msg_bits_P": P, "gadget": [bl, lv, grp]},
        "parity": {"outputs_checked": B, "decrypt_equal_lut": exact, "oracle": oracle},
        "roofline": {"kernel": k["kernel"], "bound": "f64-valu", "achieved": round(tf, 3),
                     "peak": F64_VALU_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": round(tf / F64_VALU_PEAK_TFLOPS, 4),
                     "traffic": k["hbm_bytes_per_launch"], "flops_per_launch": k["f64_flops_per_launch"],
                     "flops_source": k["flops_source"], "avg_launch_ms": k["avg_launch_ms"],
                     "launches": k["launches"], "cts_per_launch": k["cts_per_launch"],
                     "clock_mhz": k["clock_mhz"],
                     "frac_at_clock": round(tf / (F64_VALU_PEAK_TFLOPS * k["clock_mhz"] / PEAK_CLOCK_MHZ), 4)
                     if k["clock_mhz"] else None,
                     "time_source": "HIP events on the step's launches"},
        "keyswitch_ms_per_launch": round(ks["total_ms"] / max(ks["launches"], 1), 4),
        "sign_path_kernel": {"kernel": sign_kernel, "avg_launch_ms": round(sign_ms, 4),
                             "table_over_sign": round(k["avg_launch_ms"] / sign_ms, 4) if sign_ms else None},
    }
    if oracle.get("cpu_baseline"):
        line["cpu_baseline"] = oracle.pop("cpu_baseline")
    print(json.dumps(line), flush=True)


def corpus_main(args, world, rank, local, dev):
    """--mode corpus: one query against a stored corpus of encrypted
    documents (fheicp.corpus). The documents are encrypted
    before the timed region (they are persisted ciphertexts) and resident in
    HBM as seeded LWEs (D body words + 1 stream id per document). One step =
    query plan (host, D values) -> seeded linear (masks regenerated in
    registers) -> decrypt -> sign extraction -> decrypt bit -> top-k (+ the
    RCCL all-gather for N > 1)."""
    from fheicp.corpus import CorpusQuant, EncryptedCorpus
    from fheicp.datagen import training_embeddings
    from fheicp.params import sign_pbs_count
    from fheicp.search import sharded_topk
    model = build_model(args)
    e1, e2 = training_embeddings(args.dim, 1000, seed=args.seed + 1)
    cq = CorpusQuant.calibrate(model.qparams, np.concatenate([e1, e2]))
    c = EncryptedCorpus(cq).compile(key_seed=args.seed, device=local, noise_seed=args.seed + 7)
    eng = c.engine
    q_np, docs_np, base_idx = shard(args, rank, world)
    B = docs_np.shape[0]
    ids = (np.arange(B, dtype=np.uint64) + np.uint64(base_idx)) * np.uint64(args.dim)
    bodies, ids = c.encrypt_docs(docs_np, ids)
    bd = torch.from_numpy(bodies.view(np.int64)).to(dev)
    idd = torch.from_numpy(ids.view(np.int64)).to(dev)
    _, _, _, P = c.query_plan(q_np, args.min_similarity)
    p = eng.params.with_msg_bits(P)
    n_pbs = sign_pbs_count(p)

    def step():
        acc, below, _ = c.compare(bd, idd, q_np, args.min_similarity)
        oa, oi = sharded_topk(acc, below, args.top_k, base_idx, eng.topk, world)
        return acc, below, oa, oi

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    eng.profile(True)
    if dist_on():
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        acc, below, oa, oi = step()
    torch.cuda.synchronize()
    if dist_on():
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    eng.profile(False)
    br = read_br(eng)
    ks = eng.profile_read("keyswitch")
    if dist_on():
        on_dev = torch.distributed.get_backend() == "nccl"
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if on_dev else "cpu")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    value = world * B * args.steps / elapsed
    out = {
        "metric": METRIC + " [encrypted-corpus mode]",
        "value": round(value, 2), "unit": "compares/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
        "config": {
            "workload": f"search 1 clear query x {B} stored encrypted docs (seeded LWE) per GPU, {args.dim}-dim, "
                        f"n_bits={args.n_bits}, bilinear quantisation (DESIGN.md §7.1) + encrypted threshold "
                        f"(min_similarity {args.min_similarity}) + top-{args.top_k}",
            "docs_per_gpu": B, "dim": args.dim, "n_bits": args.n_bits, "n_e": cq.n_e, "P0": c.P0,
            "msg_bits_P": P, "pbs_per_compare": n_pbs, "keyswitch_per_compare": n_pbs,
            "corpus_bytes_per_doc": 8 * (args.dim + 1), "params": p.as_dict(), "parallelism": f"shard{world}",
        },
        "pbs_per_sec": round(value * n_pbs, 1),
        "roofline": roofline(p, br, B),
        "keyswitch_ms_total": round(ks["total_ms"], 3),
    }
    if rank == 0:
        from oracle import quant_ref as Q
        X, y = __import__("fheicp.datagen", fromlist=["x"]).training_pairs(args.dim, 1000, seed=args.seed + 1)
        oq = Q.fit_quantized_linear(X, y, args.n_bits)
        all_docs = np.concatenate([shard(args, r, world)[1] for r in range(world)])
        want = Q.corpus_search(oq, cq.s_e, cq.n_e, q_np, all_docs, args.top_k, args.min_similarity)
        s = np.float64(cq.out_scale)
        got = [(int(i), float(s * np.float64(a))) for a, i in zip(oa.cpu().tolist(), oi.cpu().tolist()) if i >= 0]
        ref_acc = Q.corpus_accumulate(oq, cq.s_e, cq.n_e, q_np, docs_np)
        sc = s * ref_acc.astype(np.float64)
        out["parity"] = {
            "compares_checked": B,
            "acc_bit_exact": bool(np.array_equal(acc.cpu().numpy(), ref_acc)),
            "threshold_bit_exact": bool(np.array_equal(below.cpu().numpy(), (sc < args.min_similarity).astype(np.int64))),
            "topk_equal": got == want,
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = corpus_cpu_leg(args, c, bodies, ids, oq, cq, q_np, docs_np, P, out["parity"])
        print(json.dumps(out), flush=True)
    if dist_on():
        torch.distributed.destroy_process_group()


def corpus_cpu_leg(args, c, bodies, ids, oq, cq, q_np, docs_np, P, parity):
    """The exact C oracle on a bounded sample of the corpus workload: expand
    the seeded documents, linear, decrypt, sign extraction, decrypt."""
    from oracle import quant_ref as Q
    from oracle import tfhe_ref as R
    p0 = c.scheme.as_dict()
    ref = R.RefTFHE(p0, args.seed)
    Wr, cst, T, P = c.query_plan(q_np, args.min_similarity)
    Cn = cpu_sample(args, c.scheme.with_msg_bits(P))
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    t0 = time.perf_counter()
    ct = ref.expand_seeded(bodies[:Cn], ids[:Cn], c.mask_key)
    ref.with_msg_bits(P)
    lin = ref.linear(ct, Cn, args.dim, Wr, cst - T)
    v = ref.decrypt_ints(lin)
    bits = ref.decrypt_bits(ref.sign_extract(lin))
    t_total = time.perf_counter() - t0
    acc_ref = Q.corpus_accumulate(oq, cq.s_e, cq.n_e, q_np, docs_np[:Cn])
    parity["cpu_oracle_acc_matches"] = bool(np.array_equal(v + T, acc_ref))
    parity["cpu_oracle_threshold_matches"] = bool(np.array_equal(bits, (acc_ref < T).astype(np.int64)))
    return {"value": round(Cn / t_total, 4), "unit": "compares/s", "cores": cores, "kind": "port",
            "sample": f"{Cn} compares of the same corpus workload on the exact C oracle (OpenMP {cores} threads): "
                      f"expand seeded docs + linear + decrypt + {R.sign_pbs_count(dict(p0, msg_bits=P))} KS+PBS "
                      f"sign extraction + decrypt",
            "seconds": round(t_total, 2)}


BF16_MFMA_PEAK_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md; no sparsity)
F32_MFMA_PEAK_TFLOPS = 157.3     # MI355X f32-input MFMA (v_mfma_f32_32x32x2_f32), MI355X_MICROARCH.md
# agreement with torch's fp32 forward, as tests/test_gpu_bert.py states it
EMBED_TOL = {"f32": {"cos": 1 - 1e-9, "max": 2e-4}, "bf16": {"cos": 0.99997, "max": 0.05}}


def embed_main(args, world, rank, local, dev):
    """--mode embed: the embedding stage's encoder (fheicp.bert.GpuBert, the
    forward of bert_embeddings.py:102-158) on a randomly initialised
    bert-base (the weights are an offline download; synthetic token ids,
    every sequence --seq-len tokens). One step = one forward pass + mean
    pooling of --embed-batch sequences, in --embed-precision (f32, the
    reference's arithmetic, by default). Roofline: the MFMA GEMMs
    (algorithmic 2*M*N*K per launch over their HIP-event time) against the
    dense peak of that arithmetic (f32-input or bf16 MFMA); the CPU baseline
    is the reference's own torch fp32 forward on the host cores, on a
    bounded sample."""
    from transformers import BertConfig, BertModel
    from fheicp.bert import GpuBert
    torch.manual_seed(args.seed)
    m = BertModel(BertConfig(), add_pooling_layer=False).eval()
    prec = args.embed_precision
    g = GpuBert(model=m, device=local, precision=prec)
    peak = F32_MFMA_PEAK_TFLOPS if prec == "f32" else BF16_MFMA_PEAK_TFLOPS
    B, S = args.embed_batch, args.seq_len
    gen = torch.Generator().manual_seed(args.seed + rank)
    ids = torch.randint(1000, 30000, (B, S), generator=gen)
    ids[:, 0] = 101
    ids[:, -1] = 102
    mask = torch.ones_like(ids)
    ids_d, mask_d = ids.to(dev, torch.int32), mask.to(dev, torch.int32)
    for _ in range(args.warmup):
        g.forward(ids_d, mask_d)
    torch.cuda.synchronize()
    g.profile(True)
    if dist_on():
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = g.forward(ids_d, mask_d)
    torch.cuda.synchronize()
    if dist_on():
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    g.profile(False)
    prof = {k: g.profile_read(k) for k in ("gemm", "attention", "other")}
    if dist_on():
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    seqs = world * B * args.steps
    gm = prof["gemm"]
    tf = gm["flops"] / (gm["total_ms"] * 1e-3) / 1e12 if gm["total_ms"] else 0.0
    # agreement with the fp32 torch forward on the first sequences (tolerance: tests/test_gpu_bert.py)
    n_chk = min(4, B)
    with torch.no_grad():
        ref = m(input_ids=ids[:n_chk], attention_mask=mask[:n_chk]).last_hidden_state.mean(1).double()
    got = out[:n_chk].cpu().double()
    cos = float(torch.nn.functional.cosine_similarity(got, ref, dim=1).min())
    mxd = float((got - ref).abs().max())
    tol = EMBED_TOL[prec]
    out_line = {
        "metric": "BERT embeddings/sec (encoder forward + mean pooling) [embedding stage, SURVEY.md §8f-4]",
        "value": round(seqs / elapsed, 2), "unit": "sequences/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "fp32" if prec == "f32" else "bf16",
        "data": "synthetic (random-init bert-base, random ids)",
        "config": {"workload": f"bert-base forward, {B} sequences x {S} tokens per GPU, mean pooling",
                   "batch": B, "seq_len": S, "tokens_per_step": B * S * world, "parallelism": f"replicas{world}"},
        "tokens_per_sec": round(seqs * S / elapsed, 1),
        "roofline": {"bound": "mfma", "kernel": "fbert::k_gemm2_f32<EPI>" if prec == "f32" else "fbert::k_gemm3<EPI>",
                     "achieved": round(tf, 2), "peak": peak, "unit": "TFLOP/s", "frac": round(tf / peak, 4),
                     "traffic": None, "gemm_ms_per_step": round(gm["total_ms"] / args.steps, 3),
                     "gemm_launches_per_step": gm["launches"] // max(args.steps, 1),
                     "gemm_flops_per_step": gm["flops"] / max(args.steps, 1),
                     "attention_ms_per_step": round(prof["attention"]["total_ms"] / args.steps, 3),
                     "other_ms_per_step": round(prof["other"]["total_ms"] / args.steps, 3)},
        "parity": {"sequences_checked": n_chk, "min_cosine_vs_fp32_torch": round(cos, 10),
                   "max_abs_diff_vs_fp32_torch": mxd,
                   "tolerance": f"cosine >= {tol['cos']}, max |diff| <= {tol['max']} (tests/test_gpu_bert.py)",
                   "within_tolerance": cos >= tol["cos"] and mxd <= tol["max"]},
    }
    # the reference's own forward on this GPU (torch fp32 -> hipBLASLt / MIOpen,
    # bert_embeddings.py:136 with device="cuda"), same batch, after the timed
    # region: the yardstick of the HIP encoder in the same arithmetic
    import copy
    mg = copy.deepcopy(m).to(dev)
    with torch.no_grad():
        ids_g, mask_g = ids.to(dev), mask.to(dev)
        mg(input_ids=ids_g, attention_mask=mask_g)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(max(args.steps, 2)):
            mg(input_ids=ids_g, attention_mask=mask_g).last_hidden_state.mean(1)
        torch.cuda.synchronize()
        tg = (time.perf_counter() - t0) / max(args.steps, 2)
    out_line["torch_gpu_fp32"] = {"value": round(B / tg, 2), "unit": "sequences/s", "ms_per_step": round(tg * 1e3, 3),
                                  "what": "transformers BertModel fp32 forward + mean on this GPU (the reference's "
                                          "BertEmbedder with device='cuda'), same batch"}
    del mg
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cores = torch.get_num_threads()
        nb = 8
        with torch.no_grad():
            m(input_ids=ids[:2], attention_mask=mask[:2])
            t0 = time.perf_counter()
            reps = 0
            while time.perf_counter() - t0 < 10.0:
                m(input_ids=ids[:nb], attention_mask=mask[:nb])
                reps += 1
            el = time.perf_counter() - t0
        out_line["cpu_baseline"] = {"value": round(reps * nb / el, 3), "unit": "sequences/s", "cores": cores,
                                    "kind": "reference",
                                    "sample": f"{reps} x {nb} sequences of {S} tokens through the same model in torch "
                                              f"fp32 on the host (the reference's BertEmbedder forward, "
                                              f"bert_embeddings.py:136), {cores} threads"}
    if rank == 0:
        print(json.dumps(out_line), flush=True)
    if dist_on():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
