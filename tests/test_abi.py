"""CPU: the C-ABI library loads, exports every symbol include/fhe_icp.h
declares, validates parameters and fails loudly without a device. No compute
calls (there is no GPU here)."""
import ctypes as C
import re
from pathlib import Path

import pytest

from fheicp import _lib
from fheicp.params import TOY, params_for_bits, sign_plan

INCLUDE = Path(__file__).resolve().parents[1] / "include"
HEADERS = sorted(INCLUDE.glob("*.h"))       # fhe_icp.h (the compare path), fhe_bert.h (§8 f4)


def declared_functions():
    names = set()
    for h in HEADERS:
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        names |= set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(fhe_[a-z_0-9]+)\s*\(", text, flags=re.M))
    return sorted(names)


def test_header_declares_expected_surface():
    names = declared_functions()
    for must in ("fhe_ctx_create", "fhe_keygen", "fhe_encrypt_batch", "fhe_linear_batch", "fhe_keyswitch_batch",
                 "fhe_pbs_batch", "fhe_bit_extract_batch", "fhe_decrypt_batch", "fhe_compare_batch", "fhe_topk"):
        assert must in names


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    for name in declared_functions():
        assert hasattr(L, name), name
    # and the Python binding covers all of them
    bound = {n for n, _, _ in _lib.SIGNATURES}
    assert set(declared_functions()) <= bound


def test_sizes_match_oracle(oracle_lib):
    L = _lib.lib()
    for p in (TOY, params_for_bits(16), params_for_bits(21), params_for_bits(26)):
        P = _lib.params_struct(p.as_dict())
        R = oracle_lib.RefParams(**p.as_dict())
        ol = oracle_lib.lib()
        assert L.fhe_bsk_words(C.byref(P)) == ol.ref_bsk_words(C.byref(R))
        assert L.fhe_ksk_words(C.byref(P)) == ol.ref_ksk_words(C.byref(R))
        assert L.fhe_big_lwe_words(C.byref(P)) == p.k * p.N + 1
        assert L.fhe_small_lwe_words(C.byref(P)) == p.n + 1


def test_host_context_and_validation():
    L = _lib.lib()
    P = _lib.params_struct(params_for_bits(16).as_dict())
    h = C.c_void_p()
    assert L.fhe_ctx_create(C.byref(P), -1, C.byref(h)) == 0 and h.value
    got = _lib.FheParams()
    assert L.fhe_get_params(h, C.byref(got)) == 0 and got.n == 887 and got.msg_bits == 16
    assert L.fhe_set_msg_bits(h, 60) == -1
    assert b"msg_bits" in L.fhe_last_error(h)
    # host-only contexts refuse device work with a clear error
    assert L.fhe_keygen(h, 1, None) == -2
    assert b"host-only" in L.fhe_last_error(h)
    L.fhe_ctx_destroy(h)
    bad = dict(params_for_bits(16).as_dict(), N=1000)
    Pb = _lib.params_struct(bad)
    assert L.fhe_ctx_create(C.byref(Pb), -1, C.byref(h)) == -1
    assert b"N must be" in L.fhe_last_error(None)


def test_engine_refuses_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from fheicp.engine import Engine
    with pytest.raises(_lib.FheError):
        Engine(TOY, 0)


def test_fast_gadget_validation_and_host_calls():
    """The fast-gadget fields: a fast2 gadget needs a fast one, each pair is
    all-or-nothing; fhe_sign_plan tolerates NULL outputs; a host-only context
    refuses to export a fast key."""
    L = _lib.lib()
    h = C.c_void_p()
    base = params_for_bits(19).as_dict()
    for bad, why in ((dict(base, pbs_fast_base_log=0, pbs_fast_level=0), b"fast2"),
                     (dict(base, pbs_fast2_level=0), b"fast2"),
                     (dict(base, pbs_fast_level=0), b"fast pbs")):
        P = _lib.params_struct(bad)
        assert L.fhe_ctx_create(C.byref(P), -1, C.byref(h)) == -1, bad
        assert why in L.fhe_last_error(None), L.fhe_last_error(None)
        assert L.fhe_sign_plan(C.byref(P), None, None, None) == -1
    P = _lib.params_struct(base)
    assert L.fhe_sign_plan(C.byref(P), None, None, None) == 0
    j1 = C.c_int32()
    # P = 19: a multi-bit mid gadget at the main gadget's level takes the
    # first round, so the main gadget runs none (params.sign_plan agrees)
    assert L.fhe_sign_plan(C.byref(P), None, C.byref(j1), None) == 0
    assert j1.value == sign_plan(params_for_bits(19))[1] == 0
    assert L.fhe_ctx_create(C.byref(P), -1, C.byref(h)) == 0
    buf = (C.c_uint64 * 1)()
    assert L.fhe_export_fast_bsk(h, 1, buf) == -2
    L.fhe_ctx_destroy(h)


def test_build_info_and_kernel_names_on_host_context():
    """The shipped build says ab=0; a host-only context has no launched
    kernels (empty names), rejects unknown buckets, and the table bootstrap
    and threshold entries refuse without a device."""
    L = _lib.lib()
    import __graft_entry__ as G
    # the library in the tree was compiled from these very sources
    assert L.fhe_build_info() == b"libfheicp gfx950 ab=0 src=" + G.source_sha().encode()
    assert not _lib.ab_build()
    P = _lib.params_struct(params_for_bits(16).as_dict())
    h = C.c_void_p()
    assert L.fhe_ctx_create(C.byref(P), -1, C.byref(h)) == 0
    buf = C.create_string_buffer(64)
    for k in (b"blind_rotate", b"blind_rotate_main", b"blind_rotate_fast", b"blind_rotate_fast2",
              b"blind_rotate_mid", b"blind_rotate_mid2", b"blind_rotate_mid0", b"keyswitch"):
        assert L.fhe_profile_kernel_name(h, k, buf, 64) == 0 and buf.value == b""
    assert L.fhe_profile_kernel_name(h, b"nope", buf, 64) == -1
    assert L.fhe_profile_kernel_name(h, b"keyswitch", None, 64) == -1
    assert L.fhe_pbs_table_batch(h, None, 0, None, 4, None, None) == -2
    assert L.fhe_threshold_batch(h, None, 0, 0, None, None) == -2
    assert L.fhe_debug_v4_stamps(h, buf) == -2
    assert L.fhe_debug_el_stamps(h, buf) == -2
    L.fhe_ctx_destroy(h)


def test_mid_gadget_validation_and_schedule(oracle_lib):
    """The mid-gadget fields: each pair all-or-nothing, mid needs the fast
    gadget, mid2 and mid0 need mid; fhe_sign_schedule fills at most cap
    entries and returns R; the mid keys' sizes (which = 3, 4, 5) equal the
    oracle's."""
    from fheicp.params import sign_schedule
    L = _lib.lib()
    h = C.c_void_p()
    base = params_for_bits(26).as_dict()
    assert base["pbs_mid_level"] and base["pbs_mid2_level"] and base["pbs_mid0_level"]
    for bad, why in ((dict(base, pbs_mid_level=0), b"mid pbs"),
                     (dict(base, pbs_mid_base_log=0, pbs_mid_level=0), b"mid2"),
                     (dict(base, pbs_mid2_base_log=0), b"mid2"),
                     (dict(base, pbs_mid0_level=0), b"mid0"),
                     (dict(base, pbs_mid0_group=3), b"pbs_mid0_group"),
                     (dict(base, pbs_mid_base_log=0, pbs_mid_level=0, pbs_mid2_base_log=0, pbs_mid2_level=0),
                      b"mid0"),
                     (dict(base, pbs_fast_base_log=0, pbs_fast_level=0, pbs_fast2_base_log=0, pbs_fast2_level=0),
                      b"mid pbs")):
        P = _lib.params_struct(bad)
        assert L.fhe_ctx_create(C.byref(P), -1, C.byref(h)) == -1, bad
        assert why in L.fhe_last_error(None), L.fhe_last_error(None)
        assert L.fhe_sign_schedule(C.byref(P), None, 0) == -1
    P = _lib.params_struct(base)
    R = L.fhe_sign_schedule(C.byref(P), None, 0)
    want = sign_schedule(params_for_bits(26))[1]
    assert R == len(want) == 13
    out = (C.c_int32 * 4)(-1, -1, -1, -1)
    assert L.fhe_sign_schedule(C.byref(P), out, 3) == R and list(out) == want[:3] + [-1]
    ol = oracle_lib.lib()
    RP = oracle_lib.RefParams(**base)
    for which in (1, 2, 3, 4, 5):
        assert L.fhe_fast_bsk_words(C.byref(P), which) == ol.ref_bsk2_words(C.byref(RP), which) > 0, which
    assert L.fhe_fast_bsk_words(C.byref(P), 6) == 0
    assert L.fhe_ctx_create(C.byref(P), -1, C.byref(h)) == 0
    buf = (C.c_uint64 * 1)()
    assert L.fhe_export_fast_bsk(h, 3, buf) == -2
    L.fhe_ctx_destroy(h)


def test_bert_abi_validation():
    """fhe_bert_create (include/fhe_bert.h) rejects configs the encoder does
    not implement (head dim != 64, sequences beyond 512) and, on a host with
    no device, fails with FHE_E_DEVICE instead of running anything."""
    from fheicp.bert import BertConfigC
    L = _lib.lib()
    good = dict(vocab_size=30522, hidden_size=768, num_layers=12, num_heads=12, intermediate_size=3072,
                max_position=512, type_vocab_size=2, layer_norm_eps=1e-12)
    h = C.c_void_p()
    for bad in (dict(good, num_heads=8), dict(good, max_position=1024), dict(good, hidden_size=770),
                dict(good, intermediate_size=3000), dict(good, layer_norm_eps=0.0)):
        assert L.fhe_bert_create(C.byref(BertConfigC(**bad)), 0, C.byref(h)) == -1, bad
    assert L.fhe_bert_create(C.byref(BertConfigC(**good)), 0, C.byref(h)) == -2   # no GPU here
    assert L.fhe_bert_ready(None) == 0


def test_gadget_group_validation():
    """Every gadget's grouping factor (fast, fast2, mid, mid2, mid0) is 0, 1 or 2,
    and a multi-bit (group 2) gadget needs N = 1024, k = 2, n <= 1023 and
    level <= 8 (the 48-bit-accumulator kernels go to level 8); the oracle
    library resolves the same plan for the planner's multi-bit mids."""
    from dataclasses import replace
    L = _lib.lib()
    h = C.c_void_p()
    p21 = params_for_bits(21)
    assert (p21.pbs_mid_group, p21.pbs_mid2_group) == (2, 2)
    P = _lib.params_struct(p21.as_dict())
    assert L.fhe_ctx_create(C.byref(P), -1, C.byref(h)) == 0
    L.fhe_ctx_destroy(h)
    for field in ("pbs_fast_group", "pbs_fast2_group", "pbs_mid_group", "pbs_mid2_group", "pbs_mid0_group"):
        P = _lib.params_struct(dict(p21.as_dict(), **{field: 3}))
        assert L.fhe_ctx_create(C.byref(P), -1, C.byref(h)) == -1, field
        assert b"must be 0, 1 or 2" in L.fhe_last_error(None)
    toy_mid = replace(TOY, msg_bits=11, pbs_base_log=12, pbs_level=3, pbs_fast_base_log=8, pbs_fast_level=2,
                      pbs_mid_base_log=10, pbs_mid_level=2, pbs_mid_group=2)
    P = _lib.params_struct(toy_mid.as_dict())
    assert L.fhe_ctx_create(C.byref(P), -1, C.byref(h)) == -1
    assert b"multi-bit blind rotation (group 2) needs N = 1024" in L.fhe_last_error(None)
    deep = dict(p21.as_dict(), pbs_mid_base_log=4, pbs_mid_level=9)
    P = _lib.params_struct(deep)
    assert L.fhe_ctx_create(C.byref(P), -1, C.byref(h)) == -1


def test_every_planned_parameter_set_validates():
    """params_for_bits(P) for every supported width (msg_bits >= 2) yields a
    set the library accepts (host context), with the same sign plan as
    params.py."""
    L = _lib.lib()
    h = C.c_void_p()
    for P in range(2, 28):
        p = params_for_bits(P)
        cp = _lib.params_struct(p.as_dict())
        assert L.fhe_ctx_create(C.byref(cp), -1, C.byref(h)) == 0, (P, L.fhe_last_error(None))
        L.fhe_ctx_destroy(h)
        if P >= 4:
            sched = (C.c_int32 * 64)()
            R = L.fhe_sign_schedule(C.byref(cp), sched, 64)
            from fheicp.params import sign_schedule
            assert list(sched[:R]) == sign_schedule(p)[1], P


def test_multibit_digit_width_validation():
    """Multi-bit gadgets read their digits as 32-bit fields in the 48-bit
    kernel: base_log > 31 is refused at context creation (host-only contexts
    validate too); the classic rotation and narrower multi-bit gadgets pass."""
    L = _lib.lib()
    h = C.c_void_p()
    base = params_for_bits(16).as_dict()
    P = _lib.params_struct(dict(base, pbs_fast2_base_log=32, pbs_fast2_level=1, pbs_fast2_group=2))
    assert L.fhe_ctx_create(C.byref(P), -1, C.byref(h)) == -1
    assert b"base_log <= 31" in L.fhe_last_error(None)
    assert L.fhe_sign_pbs_count(C.byref(P)) == -1
    for ok in (dict(base, pbs_fast2_base_log=31, pbs_fast2_level=1, pbs_fast2_group=2),
               dict(base, pbs_fast_base_log=16, pbs_fast_level=2, pbs_fast_group=2)):
        P = _lib.params_struct(ok)
        assert L.fhe_ctx_create(C.byref(P), -1, C.byref(h)) == 0 and h.value
        L.fhe_ctx_destroy(h)


def test_wide_multibit_and_ks_coin_bounds():
    """Two parameter bounds checked at context creation (host-only contexts
    validate too): a multi-bit gadget on the 48-bit accumulators needs
    level * base_log <= 47 (its digit fields and rounding bit live in bits
    16-63), and the key switch's tie coins must sit above every shift of the
    sign extraction: ks_level * (ks_base_log + 1) + msg_bits <= 64."""
    L = _lib.lib()
    h = C.c_void_p()
    base = params_for_bits(16).as_dict()
    for bad, msg in ((dict(base, pbs_mid_base_log=12, pbs_mid_level=4, pbs_mid_group=2), b"<= 47"),
                     (dict(base, ks_base_log=7, ks_level=7, msg_bits=16), b"msg_bits must be <= 64")):
        P = _lib.params_struct(bad)
        assert L.fhe_ctx_create(C.byref(P), -1, C.byref(h)) == -1
        assert msg in L.fhe_last_error(None), L.fhe_last_error(None)
    for ok in (dict(base, pbs_mid_base_log=15, pbs_mid_level=3, pbs_mid_group=2),
               dict(base, ks_base_log=7, ks_level=6, msg_bits=16)):
        P = _lib.params_struct(ok)
        assert L.fhe_ctx_create(C.byref(P), -1, C.byref(h)) == 0 and h.value
        L.fhe_ctx_destroy(h)


def test_gemm_lds_dma_pipelines_not_drained():
    """ISA lint (no GPU): every BERT GEMM instantiation keeps its LDS-DMA
    pipeline: no vmcnt(0) between the next step's global_load_lds and the
    current step's first ds_read (tools/isa_lint.py)."""
    import shutil
    import subprocess
    import sys
    from pathlib import Path
    if not shutil.which("hipcc"):
        pytest.skip("no hipcc")
    repo = Path(__file__).resolve().parents[1]
    r = subprocess.run([sys.executable, str(repo / "tools" / "isa_lint.py")], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr[-2000:]
    assert r.stdout.count("k_gemm") >= 6


def test_params_struct_size_refuses_stale_bindings():
    """fhe_params leads with struct_size, checked by every entry
    point that validates parameters. A binding built against the previous
    header (no struct_size, 26 fields) puts n = 887 in its place and is
    refused with FHE_E_ARG instead of read past its end; the Python binding's
    field list is the header's."""
    import re
    hdr = (Path(__file__).resolve().parents[1] / "include" / "fhe_icp.h").read_text()
    body = re.search(r"typedef struct fhe_params \{(.*?)\} fhe_params;", hdr, re.S).group(1)
    fields = re.findall(r"int32_t\s+(\w+);", body)
    assert fields == ["struct_size"] + list(_lib.PARAM_FIELDS)
    L = _lib.lib()
    assert C.sizeof(_lib.FheParams) == 4 * len(fields)

    class Old(C.Structure):
        _fields_ = [(f, C.c_int32) for f in _lib.PARAM_FIELDS]
    d = params_for_bits(16).as_dict()
    old = Old(**{f: int(d.get(f, 0)) for f in _lib.PARAM_FIELDS})
    h = C.c_void_p()
    assert L.fhe_ctx_create(C.cast(C.byref(old), C.POINTER(_lib.FheParams)), -1, C.byref(h)) == -1
    assert b"struct_size" in L.fhe_last_error(None)
    assert L.fhe_sign_pbs_count(C.cast(C.byref(old), C.POINTER(_lib.FheParams))) == -1
    P = _lib.params_struct(d)
    assert P.struct_size == C.sizeof(_lib.FheParams)
    assert L.fhe_ctx_create(C.byref(P), -1, C.byref(h)) == 0
    got = _lib.FheParams()
    assert L.fhe_get_params(h, C.byref(got)) == 0 and got.struct_size == P.struct_size
    L.fhe_ctx_destroy(h)


def test_table_gadget_matches_params():
    """fhe_pbs_table_gadget (the gadget the table bootstrap runs on) agrees
    with params.table_gadget on every planned width and TOY: (15,2) multi-bit
    at P = 16, mid0 (5,8) at P = 26, the classic main gadget on TOY."""
    from fheicp.params import table_gadget
    L = _lib.lib()
    for P in list(range(4, 28)):
        p = params_for_bits(P)
        cp = _lib.params_struct(p.as_dict())
        assert L.fhe_pbs_table_gadget(C.byref(cp)) == table_gadget(p), P
    assert table_gadget(params_for_bits(16)) == 1
    assert table_gadget(params_for_bits(26)) == 5
    assert L.fhe_pbs_table_gadget(C.byref(_lib.params_struct(TOY.as_dict()))) == table_gadget(TOY) == 0
    bad = _lib.params_struct(dict(TOY.as_dict(), N=1000))
    assert L.fhe_pbs_table_gadget(C.byref(bad)) == -1


def test_integration_guide_names_every_entry_point():
    """INTEGRATION.md's ABI table covers every function the headers declare
    (the guide a maintainer binds from stays in step with the library)."""
    text = (Path(__file__).resolve().parents[1] / "INTEGRATION.md").read_text()
    missing = [n for n in declared_functions() if n not in text]
    assert not missing, missing
