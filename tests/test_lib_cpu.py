"""CPU-only checks of the product boundary (no GPU calls).

* the C-ABI library loads and exports every symbol include/pt_cell.h declares;
* size queries (pure host code) behave and reject unsupported shapes;
* the drop-in model keeps the reference's state_dict keys / shapes / order,
  its initial values (same RNG order; pinned by tests/golden/init_*.npz) and
  refuses to run off-GPU instead of falling back to a CPU path.
"""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from goldens import GOLDEN, load

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols(header="pt_cell.h"):
    txt = open(os.path.join(REPO, "include", header)).read()
    return sorted(set(re.findall(r"\b(pt_[a-z0-9_]+)\s*\(", txt)))


def _bindings():
    from ptamd import _lib, lstm, readout, tfrecord
    return [("pt_cell.h", _lib, "pt_version", "pt_cell"),
            ("pt_readout.h", readout, None, None),
            ("pt_lstm.h", lstm, "pt_lstm_version", "pt_lstm"),
            ("pt_tfrecord.h", tfrecord, None, None)]


def test_header_and_binding_agree():
    for header, mod, _, _ in _bindings():
        assert sorted(mod.EXPORTS) == _header_symbols(header), header


def test_library_exports_every_symbol():
    for header, mod, ver, prefix in _bindings():
        lib = mod.load()
        for sym in _header_symbols(header):
            assert hasattr(lib, sym), (header, sym)
        if ver:
            assert getattr(lib, ver)().decode().startswith(prefix)


def test_size_queries_and_validation():
    from ptamd import _lib
    lib = _lib.load()
    d = _lib.Desc(batch=256, channels=32, frames=64, height=32, width=32, ksize=7, act=0,
                  no_inh=0, cell=0, dtype=_lib.PT_DTYPE_BF16, eps=1e-3)
    saved = lib.pt_cell_saved_bytes(ctypes.byref(d))
    frame = 256 * 1024 * 32 * 2
    assert saved >= 6 * 64 * frame          # six per-frame tensors kept for BPTT
    assert lib.pt_cell_workspace_bytes(ctypes.byref(d)) >= 2 * 64 * frame
    bad = _lib.Desc(batch=2, channels=33, frames=8, height=32, width=32, ksize=7, act=0,
                    no_inh=0, cell=0, dtype=0, eps=1e-3)
    assert lib.pt_cell_saved_bytes(ctypes.byref(bad)) == 0
    assert b"channels" in lib.pt_last_error()
    for k in (4, 17):                        # odd, <= 15 (the constructors' default is 15)
        bad.channels, bad.ksize = 32, k
        assert lib.pt_cell_saved_bytes(ctypes.byref(bad)) == 0
        assert b"ksize" in lib.pt_last_error()
    # C < 32 runs zero-padded (the padded parameter copies live in the saved blob);
    # k = 9..15 uses the 46 x 46 tile and K*K-tap weight fragments
    ok = _lib.Desc(batch=2, channels=8, frames=8, height=32, width=32, ksize=15, act=0,
                   no_inh=0, cell=0, dtype=0, eps=1e-3)
    assert lib.pt_cell_saved_bytes(ctypes.byref(ok)) > 0
    ok.channels = 32
    assert lib.pt_cell_saved_bytes(ctypes.byref(ok)) > 0
    # frames larger than 32x32 run as 32x32 tiles: sizes scale with the tile count
    # (cfg4: hGRU 64x64x128f, 128 clips per GPU); sides must be multiples of 32
    big = _lib.Desc(batch=128, channels=32, frames=128, height=64, width=64, ksize=7, act=0,
                    no_inh=0, cell=1, dtype=_lib.PT_DTYPE_BF16, eps=1e-3)
    assert lib.pt_cell_saved_bytes(ctypes.byref(big)) >= 7 * 128 * (128 * 4096 * 32 * 2)
    for h, w in ((48, 64), (64, 40), (16, 32)):
        big.height, big.width = h, w
        assert lib.pt_cell_saved_bytes(ctypes.byref(big)) == 0
        assert b"multiple of 32" in lib.pt_last_error()
    # input layouts: f32 [B,3,T,H,W] (0) or raw u8 clips [B,T,H,W,3] (1); same sizes
    d.x_format = _lib.PT_X_U8_NTHWC
    assert lib.pt_cell_saved_bytes(ctypes.byref(d)) == saved
    d.x_format = 2
    assert lib.pt_cell_saved_bytes(ctypes.byref(d)) == 0
    assert b"x_format" in lib.pt_last_error()


def test_state_split_round_trips_and_keeps_nan():
    """The bf16 cell's hi / lo split of E and I (pt_cell_split_bits: the same
    inline function the kernels' stores use): hi + sext(lo) gives
    every finite value and +-Inf back bit for bit, hi is the value rounded half
    up in magnitude, and a NaN stays NaN in hi and in hi + lo (including the
    mantissas whose half-up add would carry out of the exponent)."""
    from ptamd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(0)
    fin = (rng.standard_normal(20000) * 10.0 ** rng.integers(-40, 38, 20000)).astype(np.float32)
    special = np.array([0.0, -0.0, np.inf, -np.inf, 3.4028235e38, -3.4028235e38, 1e-45, -1e-45,
                        np.float32(1.0) + np.float32(2 ** -8), np.float32(1.0) + np.float32(2 ** -9)],
                       dtype=np.float32)
    nan_bits = np.array([0x7FC00000, 0x7FFF8000, 0x7FFFFFFF, 0xFFFF8000, 0xFFFFFFFF, 0x7F800001,
                         0x7F808000, 0xFF800001, 0x7FBFFFFF], dtype=np.uint32)
    bits = np.concatenate([fin.view(np.uint32), special.view(np.uint32), nan_bits])
    n = len(bits)
    hi = np.zeros(n, np.uint16)
    lo = np.zeros(n, np.uint16)
    assert lib.pt_cell_split_bits(bits.ctypes.data, hi.ctypes.data, lo.ctypes.data, n) == 0
    back = ((hi.astype(np.uint32) << 16) + lo.astype(np.int16).astype(np.int64).astype(np.uint32)).astype(np.uint32)
    hif = (hi.astype(np.uint32) << 16).view(np.float32)
    isn = np.isnan(bits.view(np.float32))
    assert isn.sum() == len(nan_bits)
    assert np.array_equal(back[~isn], bits[~isn])
    assert np.isnan(hif[isn]).all() and np.isnan(back.view(np.float32)[isn]).all()
    # hi: half up in magnitude (ties away from zero), i.e. the upper 16 bits of bits + 0x8000
    ref = ((bits[~isn].astype(np.uint64) + 0x8000) >> 16).astype(np.uint16)
    assert np.array_equal(hi[~isn], ref)
    assert lib.pt_cell_split_bits(None, None, None, 1) != 0


def test_u8_input_helpers_match_prepare_data():
    """The u8 input path's conversion and readout target are bit-identical to
    engine.prepare_data's f32 tensor (utils/engine.py:220-255)."""
    import types
    import numpy as np
    import torch
    from ptamd import cell, synth
    from utils import engine
    clips, labels = synth.make_batch(5, 3, 4, h=32, w=32)
    args = types.SimpleNamespace(pretrained=False)
    x, y = engine.prepare_data(clips, labels, args, "cpu", False)
    xu, yu = engine.prepare_data(clips, labels, args, "cpu", False, keep_u8=True)
    assert xu.dtype == torch.uint8 and tuple(xu.shape) == clips.shape
    assert torch.equal(yu, y)
    assert torch.equal(cell.unit_values(xu).permute(0, 4, 1, 2, 3), x)
    assert torch.equal(cell.target_channel(xu), x[:, 2, 0])
    assert cell.clip_dims(xu) == cell.clip_dims(x) == (3, 4, 32, 32)
    # every byte value, against numpy's float64 quotient
    allv = torch.arange(256, dtype=torch.uint8)
    ref = (np.arange(256, dtype=np.float64) / 255.).astype(np.float32)
    assert np.array_equal(cell.unit_values(allv).numpy(), ref)
    # disentangle / pretrained keep the f32 path
    xd, _ = engine.prepare_data(clips, labels, args, "cpu", True, keep_u8=True)
    assert xd.dtype == torch.float32


@pytest.mark.parametrize("tag", ["int_c32", "int_noinh", "int_lesion"])
def test_state_dict_keys_match_reference(tag):
    from models import InT as int_mod
    g = load(tag)
    ref_keys = [k[len("param."):] for k in g if k.startswith("param.")]
    kw = dict(dimensions=32, timesteps=8, kernel_size=7, no_inh=bool(g["cfg_no_inh"]))
    m = int_mod.InT(**kw)
    sd = m.state_dict()
    assert list(sd) == ref_keys            # same keys, same order
    for k in ref_keys:
        assert tuple(sd[k].shape) == g["param." + k].shape, k


def test_init_matches_reference_rng_order():
    from models import InT as int_mod
    path = os.path.join(GOLDEN, "init_seed123.npz")
    if not os.path.exists(path):
        pytest.skip("init fixture not generated")
    z = np.load(path, allow_pickle=False)
    torch.manual_seed(123)
    m = int_mod.InT(dimensions=32, timesteps=8, kernel_size=7)
    sd = m.state_dict()
    for k in z.files:
        np.testing.assert_array_equal(sd[k].numpy(), z[k], err_msg=k)


def test_hgru_init_and_keys_match_reference():
    """FFhGRU drop-in: state_dict keys in the reference order and the initial
    values under seed 123 bit-identical (models/ffhgru_hierarchy.py:58-207)."""
    from models import ffhgru_hierarchy as hg
    z = np.load(os.path.join(GOLDEN, "init_hgru_seed123.npz"), allow_pickle=False)
    torch.manual_seed(123)
    m = hg.FFhGRU(dimensions=32, timesteps=8, kernel_size=7)
    sd = m.state_dict()
    assert [k for k in sd if k != "unit1.w"] == list(z.files)
    for k in z.files:
        np.testing.assert_array_equal(sd[k].numpy(), z[k], err_msg=k)
    g = np.load(os.path.join(GOLDEN, "hgru_c32.npz"), allow_pickle=False)
    assert list(sd) == [k[len("param."):] for k in g.files if k.startswith("param.")]


def test_lesion_freezes_only_named_params():
    from models import InT as int_mod
    m = int_mod.InT(dimensions=32, kernel_size=7, lesion_alpha=True, lesion_gamma=True)
    frozen = {n for n, p in m.named_parameters() if not p.requires_grad}
    assert frozen == {"unit1.alpha", "unit1.gamma"}


def test_no_cpu_fallback():
    from models import InT as int_mod
    m = int_mod.InT(dimensions=32, timesteps=4, kernel_size=7)
    with pytest.raises(RuntimeError, match="ROCm device"):
        m(torch.rand(1, 3, 4, 32, 32))


def test_lstm_size_queries_and_validation():
    from ptamd import lstm
    lib = lstm.load()
    d = lstm.Desc(batch=256, in_channels=25, channels=25, height=32, width=32, ksize=15,
                  steps=8, dtype=lstm.PT_LSTM_BF16, init_state=0)
    saved = lib.pt_lstm_saved_bytes(ctypes.byref(d))
    step = 256 * 1024
    assert saved >= 8 * step * (128 * 4 + 32 * 2 + 32 * 4)   # P_t, h_t, c_t per step
    assert lib.pt_lstm_workspace_bytes(ctypes.byref(d)) >= 8 * step * 128 * 2
    for field, val, msg in (("ksize", 4, b"ksize"), ("ksize", 17, b"ksize"),
                            ("channels", 33, b"hidden"), ("height", 64, b"32x32"),
                            ("steps", 0, b"steps")):
        bad = lstm.Desc(batch=2, in_channels=25, channels=25, height=32, width=32, ksize=7,
                        steps=4, dtype=0, init_state=0)
        setattr(bad, field, val)
        assert lib.pt_lstm_saved_bytes(ctypes.byref(bad)) == 0, field
        assert msg in lib.pt_lstm_last_error(), (field, lib.pt_lstm_last_error())
    # the clip stem validates before touching the device (dummy pointers)
    assert lib.pt_lstm_stem_workspace_bytes(3) == 1024 * 32 * 4 * 4
    assert lib.pt_lstm_stem_workspace_bytes(5) == 0
    dummy = ctypes.c_void_p(16)
    for cin, cout, n, msg in ((5, 25, 1024, b"cin 1..4"), (3, 33, 1024, b"cout 1..32"),
                              (3, 25, 1022, b"multiple of 4")):
        rc = lib.pt_lstm_stem_forward(dummy, 0, dummy, dummy, 2, cin, cout, n, dummy, None)
        assert rc == lstm.PT_LSTM_ERR_UNSUPPORTED and msg in lib.pt_lstm_last_error(), msg


def test_convlstm_keys_and_init_match_reference():
    """ConvLSTM drop-in: state_dict keys in the reference order (convlstm.py:93-114)
    and initial values under seed 123 bit-identical (Gabor conv0, RNG order)."""
    from models import convlstm as cl
    z = np.load(os.path.join(GOLDEN, "init_convlstm_seed123.npz"), allow_pickle=False)
    torch.manual_seed(123)
    m = cl.ConvLSTM(timesteps=4, filt_size=7)
    sd = m.state_dict()
    assert list(sd) == list(z.files)
    for k in z.files:
        np.testing.assert_array_equal(sd[k].numpy(), z[k], err_msg=k)
    g = np.load(os.path.join(GOLDEN, "convlstm_k15.npz"), allow_pickle=False)
    m15 = cl.ConvLSTM(timesteps=3, filt_size=15)
    assert list(m15.state_dict()) == [k[len("param."):] for k in g.files if k.startswith("param.")]


def test_convlstm_no_cpu_fallback():
    from models import convlstm as cl
    m = cl.ConvLSTM(timesteps=2, filt_size=7)
    with pytest.raises(RuntimeError, match="ROCm device"):
        m(torch.rand(1, 1, 32, 32), 0, 0, torch.zeros(1, 32, 32, dtype=torch.long),
          torch.nn.CrossEntropyLoss())


@pytest.mark.parametrize("dtype", [torch.float64, torch.bfloat16])
def test_param_staging_cache_reuses_its_buffer(dtype):
    """Non-f32 parameters are staged into ONE persistent f32 buffer per
    parameter (stable device pointers for the cached hipGraph): a second
    lookup must return the same buffer, refreshed, not raise (a tensor-keyed
    WeakKeyDictionary compares keys element-wise)."""
    from ptamd.cell import _as_f32
    p = torch.nn.Parameter(torch.randn(5, 3, dtype=dtype))
    a = _as_f32(p)
    b = _as_f32(p)
    assert a is b and a.dtype == torch.float32
    with torch.no_grad():
        p.add_(1)
    c = _as_f32(p)
    assert c is a and torch.equal(c, p.detach().float())


def test_release_library_has_no_diagnostic_switches():
    """The release libptcell.so never reads PT_CELL_ABLATE / PT_CELL_DEBUG_STOP
    (compiled only into libptcell_diag.so, -DPT_DIAG=1) and refuses
    pt_cell_trace, so a stray environment variable cannot alter training;
    the diagnostic build keeps them for tools/ (host calls only, no GPU)."""
    from ptamd import _lib
    rel = open(_lib.LIB_PATH, "rb").read()
    diag = open(_lib.DIAG_PATH, "rb").read()
    for name in (b"PT_CELL_ABLATE", b"PT_CELL_DEBUG_STOP"):
        assert name not in rel, name
        assert name in diag, name
    lib = _lib.load()
    assert "diag" not in lib.pt_version().decode()
    assert lib.pt_cell_trace(None, -1) == 2          # PT_ERR_UNSUPPORTED
    assert b"diagnostic build" in lib.pt_last_error()
    dl = ctypes.CDLL(_lib.DIAG_PATH)
    dl.pt_version.restype = ctypes.c_char_p
    assert "diag" in dl.pt_version().decode()
    dl.pt_cell_trace.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert dl.pt_cell_trace(None, -1) == 0


# the kernel-variant switches (PT_SW, csrc/pt_device.h): A/B experiments of
# DESIGN.md §9, read only by the diagnostic builds
CELL_SWITCHES = (b"PT_CELL_FUSED", b"PT_PWB2", b"PT_PWA2", b"PT_WG16", b"PT_WGDMA", b"PT_CELL_PERSIST",
                 b"PT_XCD_MAP", b"PT_CONV_BAND", b"PT_CPA", b"PT_BAND2_TILED",
                 b"PT_FUSED_TILED")
LSTM_SWITCHES = (b"PT_LCONV_FAST", b"PT_LCONVT8", b"PT_LWGRAD2", b"PT_LPW_FUSE")


def test_release_libraries_freeze_the_kernel_variant_switches():
    """The release libptcell.so / libptlstm.so compile every kernel-variant
    switch to its default: the names are not in the binaries at all, so the
    environment cannot change which kernels run (tests/test_gpu_trace.py
    checks on the GPU that setting them all leaves the results bitwise
    unchanged).  The diagnostic builds keep them for the A/B tests
    (tests/variants.py), and diag_library() routes calls there and back."""
    from ptamd import _lib, lstm
    for rel, diag, names in ((_lib.LIB_PATH, _lib.DIAG_PATH, CELL_SWITCHES),
                             (lstm.LIB_PATH, lstm.DIAG_PATH, LSTM_SWITCHES)):
        r, d = open(rel, "rb").read(), open(diag, "rb").read()
        for name in names:
            assert name not in r, (rel, name)
            assert name in d, (diag, name)
    rel_v = _lib.load().pt_version().decode()
    with _lib.diag_library() as dl:
        assert _lib.load() is dl and "diag" in dl.pt_version().decode()
    assert _lib.load().pt_version().decode() == rel_v and "diag" not in rel_v
    with lstm.diag_library():
        assert "diag" in lstm.load().pt_lstm_version().decode()
    assert "diag" not in lstm.load().pt_lstm_version().decode()


def _listing(path):
    """The shipped gfx950 machine code of a built library as a listing
    (tools/isa_listing.py: unbundle + llvm-objdump)."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import isa_listing
    return isa_listing.listing(path).split("\n")


def _libpath(which):
    from ptamd import _lib, lstm
    return {"cell": _lib.LIB_PATH, "lstm": lstm.LIB_PATH}[which]


@pytest.mark.parametrize("which", ["cell", "lstm"])
def test_no_packed_f32_op_reads_a_register_the_previous_valu_op_wrote(which):
    """Guard for the r04 determinism fix (ptamd/build.py
    -fno-slp-vectorize): a packed-FP32 op (v_pk_fma/mul/add_f32) issued right
    after the VALU instruction that wrote the HIGH register of its source
    pair read that register stale now and then in the wave's last 16 lanes,
    so the bf16 backward differed run to run.  The release code objects must
    hold no such pair (tools/pk_hazard_scan.py logic on the disassembled .so);
    a build with the SLP vectorizer back on has hundreds."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from waitcnt_check import functions, split_ops
    from trans_hazard_scan import instrs
    from trans_src_scan import dst_of
    pk = re.compile(r"^v_pk_(fma|mul|add)_f32")
    bad, npk = [], 0
    for name, body in functions(_listing(_libpath(which)), None):
        ins = instrs(body)
        for i, s in enumerate(ins[1:], 1):
            op = s.split()[0]
            if not pk.match(op):
                continue
            npk += 1
            w = dst_of(ins[i - 1])
            for tok in split_ops(s[len(op):])[1:]:
                m = re.search(r"v\[(\d+):(\d+)\]", tok)
                if m and ("v", int(m.group(2))) in w:
                    bad.append((name[:60], ins[i - 1], s))
    assert npk > 0 or which == "lstm"     # the listing parse found the cell's explicit f32x2 math
    assert not bad, bad[:5]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("which", ["cell", "lstm"])
def test_every_load_result_is_waited_for_before_use(which):
    """tools/waitcnt_check.py on the shipped code objects: a data-flow pass
    over every kernel's basic blocks finds no instruction that touches a
    load's destination register before an s_waitcnt retired that load."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from waitcnt_check import check, functions
    nk, bad = 0, []
    for name, body in functions(_listing(_libpath(which)), None):
        nk += 1
        rep = check(body)
        if rep:
            bad.append((name[:60], len(rep), rep[0][1]))
    assert nk > 10 and not bad, bad[:5]
