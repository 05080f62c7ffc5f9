"""CPU: the C-ABI library loads and exports every declared symbol, argument validation runs
without a GPU, and the host-side logic (drop-in CrossCoder surface, checkpoints, schedules,
Buffer protocol) matches the reference."""
import ctypes
import json
import os
import re
import shutil

import numpy as np
import pytest
import torch

import crosscoder_amd as ca
from crosscoder_amd import _lib, trainer as ca_trainer
from oracle import cpu_reference as O
from tests._golden import GOLDEN, load

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "crosscoder_hip.h")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(cc_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    syms = declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert s in _lib.SIGNATURES, f"{s} declared in the header but not typed in _lib.py"
        getattr(lib, s)  # raises AttributeError if the .so does not export it
    assert set(_lib.SIGNATURES) == set(syms)
    assert lib.cc_version() >= 100


def _dynamic_exports(path):
    import shutil
    import subprocess
    nm = shutil.which("nm") or shutil.which("llvm-nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    if not os.path.exists(nm):
        pytest.skip("no nm")
    out = subprocess.run([nm, "-D", "--defined-only", path], check=True, capture_output=True, text=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_library_exports_only_the_header():
    """The product library exports exactly the C ABI of include/crosscoder_hip.h (no global-state setters, no
    kernel handles); the test-only debug build adds only its launch-form setters."""
    syms = set(declared_symbols())
    assert _dynamic_exports(_lib.LIB_PATH) == syms
    assert _dynamic_exports(_lib.DEBUG_LIB_PATH) == syms | set(_lib.DEBUG_SETTERS) | {"cc_debug_spin", "cc_debug_spin_ev",
                                                                       "cc_debug_set_stamps", "cc_debug_get_q4"}


def test_argument_validation_without_gpu():
    lib = _lib.load()
    null = ctypes.c_void_p(0)
    assert lib.cc_prep_input(null, 1, null, 1, null, null, 4, 2, 8, 1, null) == 1          # NULL
    assert lib.cc_gemm_f32out(null, 0, 8, null, 0, 8, null, 8, 8, 8, 8, 1, null) == 1        # NULL
    fake = ctypes.c_void_p(1 << 20)
    assert lib.cc_gemm_f32out(fake, 0, 8, fake, 0, 8, fake, 8, 8, 8, 8, 7, null) == 2        # dtype
    assert lib.cc_gemm_f32out(fake, 0, 12, fake, 0, 12, fake, 12, 8, 8, 12, 1, null) == 3    # K % 8
    assert lib.cc_dec_norms(fake, fake, fake, null, 8, 2, 12, 1, null) == 3                         # d % 8
    assert lib.cc_clip_finalize(fake, (ctypes.c_int64 * 2)(0, 1), 9, 1.0, 0, fake, null) == 3
    assert b"NULL" in lib.cc_strerror(1)
    assert lib.cc_col_part_rows(4096) == 32 and lib.cc_wave_parts(4096, 16384) == 8 * 16 * 64
    assert lib.cc_wgrad_parts(16384, 4608, 1) == 8 * 64 * 18  # bf16: ping-pong 256 x 256 tiles
    assert lib.cc_wgrad_parts(16384, 4608, 2) == 8 * 64 * 18  # fp32: 256 x 256 tiles
    assert lib.cc_wgrad_parts(16384, 4608, 2) == 8 * 64 * 18  # fp32: 256 x 256
    assert lib.cc_loss_col_blocks(2304) == 5
    # fused step tails (cc_grad_tail / cc_loss_tail): NULL and shape checks come before any launch
    off = (ctypes.c_int64 * 5)(0, 1, 2, 3, 4)
    assert lib.cc_grad_tail(null, 16, 256, fake, fake, fake, 128, 64, fake, fake, 1, fake, off, 4, 1.0, 1, fake, fake,
                            null) == 1
    assert lib.cc_grad_tail(fake, 16, 256, fake, fake, fake, 128, 64, fake, fake, 1, fake, off, 4, 1.0, 1, fake, null,
                            null) == 1                                                           # no counter
    assert lib.cc_grad_tail(fake, 0, 256, fake, fake, fake, 128, 64, fake, fake, 1, fake, off, 4, 1.0, 1, fake, fake,
                            null) == 3                                                           # R_enc = 0
    assert lib.cc_grad_tail(fake, 16, 256, fake, fake, fake, 128, 64, fake, fake, 1, fake, off, 9, 1.0, 1, fake, fake,
                            null) == 3                                                           # nparams > 8
    assert lib.cc_loss_tail(fake, fake, 256, fake, fake, 36, fake, 8, fake, fake, fake, fake, null, null, 0, 64, 2,
                            32, null, null) == 1                                                 # no counter
    assert lib.cc_loss_tail(null, fake, 256, fake, fake, 36, fake, 8, fake, fake, fake, fake, null, null, 0, 64, 2,
                            32, fake, null) == 1                                                 # no column sums
    assert lib.cc_loss_tail(fake, fake, 256, fake, fake, 36, fake, 8, fake, fake, fake, fake, null, null, 0, 0, 2,
                            32, fake, null) == 3                                                 # empty batch
    assert lib.cc_loss_tail(fake, fake, 256, fake, fake, 0, fake, 8, fake, fake, fake, fake, null, null, 0, 64, 2,
                            32, fake, null) == 3                                                 # ncb = 0
    assert lib.cc_loss_finalize_nb(null, 36, fake, 8, fake, 8, fake, fake, fake, fake, null, null, 0, 64, 2, 32,
                                   null) == 1
    # G2 + loss in one pass (cc_decode_loss_t): served shapes, checks before any launch
    assert lib.cc_decode_loss_ncb(4096, 16384, 2, 2304, 1) == 36      # config 2: d / 64 row-term blocks
    assert lib.cc_decode_loss_ncb(4096, 16384, 2, 2304, 2) == 0       # fp32: two-pass form
    assert lib.cc_decode_loss_ncb(4096, 16384, 2, 200, 1) == 0        # d % 64
    assert lib.cc_decode_loss_ncb(4100, 16384, 2, 2304, 1) == 0       # B % 8
    args = [fake] * 10 + [fake, 0, 4096, 16384, 2, 2304, 1, null]
    args[5] = ctypes.c_float(2.0 / 4096)
    bad = list(args)
    bad[3] = null
    assert lib.cc_decode_loss_t(*bad) == 1                            # no x
    bad = list(args)
    bad[15] = 200
    assert lib.cc_decode_loss_t(*bad) == 3                            # d % 64


def _cfg(dtype="bf16", h=256, d=32, device="cpu"):
    return {"seed": 49, "batch_size": 64, "buffer_mult": 128, "lr": 5e-5, "num_tokens": 640, "l1_coeff": 2,
            "beta1": 0.9, "beta2": 0.999, "dict_size": h, "seq_len": 1024, "enc_dtype": dtype, "device": device,
            "dec_init_norm": 0.08, "d_in": d, "log_every": 100, "save_every": 30000}


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_crosscoder_params_match_reference_layout(dtype):
    cc = ca.CrossCoder(_cfg(dtype))
    r = load(f"step_b64_n2_d32_h256_{dtype}")
    sd = cc.state_dict()
    assert list(sd.keys()) == ["W_enc", "W_dec", "b_enc", "b_dec"]
    for k, v in r["init"].items():
        assert sd[k].shape == v.shape and sd[k].dtype == v.dtype and sd[k].stride() == v.stride(), k
        assert torch.equal(sd[k], v), k
    # parameters() order = the reference's (clip / Adam iterate in this order)
    assert [p.shape for p in cc.parameters()] == [v.shape for v in r["init"].values()]


def test_loads_reference_checkpoint(tmp_path):
    src = os.path.join(GOLDEN, "ckpt", "version_0")
    cfg = json.load(open(os.path.join(src, "0_cfg.json")))
    cwd = os.getcwd()
    try:
        os.chdir(tmp_path)
        shutil.copytree(src, tmp_path / "checkpoints" / "version_0")
        cc = ca.CrossCoder.load("version_0", 0)
        ref = torch.load(os.path.join(src, "0.pt"), weights_only=True)
        for k, v in ref.items():
            assert torch.equal(cc.state_dict()[k], v), k
            assert cc.state_dict()[k].stride() == v.stride(), k
        # our save() writes the same two-file layout, reloadable by torch alone
        cc.save()
        out = tmp_path / "checkpoints" / "version_1"
        assert sorted(os.listdir(out)) == ["0.pt", "0_cfg.json"]
        sd = torch.load(out / "0.pt", weights_only=True)
        for k, v in ref.items():
            assert torch.equal(sd[k], v) and sd[k].stride() == v.stride(), k
        assert json.load(open(out / "0_cfg.json")) == cfg
    finally:
        os.chdir(cwd)


def test_load_from_hf_reads_a_local_hub_layout(tmp_path):
    """crosscoder.py:160-205 minus the download: {local_dir}/{path}/cfg.json + cc_weights.pt (the Hub repo's
    layout, e.g. blocks.14.hook_resid_pre/) loads through CrossCoder.load_from_hf(local_dir=...), the
    device override applies, and the weights / strides are the file's."""
    src = os.path.join(GOLDEN, "ckpt", "version_0")
    cfg = json.load(open(os.path.join(src, "0_cfg.json")))
    ref = torch.load(os.path.join(src, "0.pt"), weights_only=True)
    d = tmp_path / "blocks.14.hook_resid_pre"
    d.mkdir()
    json.dump(dict(cfg, device="cuda:7"), open(d / "cfg.json", "w"))  # the override must win
    torch.save(ref, d / "cc_weights.pt")
    cc = ca.CrossCoder.load_from_hf(path="blocks.14.hook_resid_pre", device="cpu", local_dir=tmp_path)
    assert cc.cfg["device"] == "cpu"
    for k, v in ref.items():
        assert torch.equal(cc.state_dict()[k], v) and cc.state_dict()[k].stride() == v.stride(), k
    with pytest.raises(RuntimeError, match="no network"):
        ca.CrossCoder.load_from_hf()


def test_arena_repacks_after_param_replacement():
    cc = ca.CrossCoder(_cfg())
    before = cc.W_dec.detach().clone()
    cc.W_dec.data = cc.W_dec.data.clone()  # breaks the arena aliasing
    a = cc.arena()
    assert a.W_dec().data_ptr() == cc.W_dec.data_ptr()
    assert torch.equal(cc.W_dec.detach(), before)
    assert cc.W_enc.stride() == (32, 1, 64)


def test_compute_refuses_cpu_tensors():
    cc = ca.CrossCoder(_cfg())
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        cc.encode(torch.zeros(4, 2, 32, dtype=torch.bfloat16))


def test_schedules_match_reference():
    r = load("step_b32_n2_d32_h128_fp32")
    cfg = r["cfg"]

    class _NoBuf:
        normalize = True

    tr = ca_trainer.Trainer.__new__(ca_trainer.Trainer)
    tr.cfg = cfg
    tr.total_steps = cfg["num_tokens"] // cfg["batch_size"]
    tr.step_counter = 0

    class _Opt:
        param_groups = [{"lr": cfg["lr"], "initial_lr": cfg["lr"]}]

    sched = ca_trainer.LambdaLRHost(_Opt(), tr.lr_lambda)
    for s, d in enumerate(r["steps"]["loss_dicts"]):
        tr.step_counter = s
        assert tr.get_l1_coeff() == d["l1_coeff"] == O.l1_coeff(s, tr.total_steps, cfg["l1_coeff"])
        sched.step()
        assert sched.get_last_lr()[0] == d["lr"]


class FakeLM:
    """Deterministic HookedTransformer stand-in (tools/gen_golden.py): table[token] + pos."""

    class _C:
        pass

    def __init__(self, table, pos):
        self.table, self.pos = table, pos
        self.cfg = FakeLM._C()
        self.cfg.d_model = table.shape[1]

    def run_with_cache(self, tokens, names_filter=None, return_type=None):
        return None, {names_filter: self.table[tokens] + self.pos[None, : tokens.shape[1]]}


def test_buffer_norm_factors_match_reference():
    """Buffer.estimate_norm_scaling_factor (buffer.py:44-63) on the fake LMs (host-side harvest
    statistics; the buffer itself is GPU-resident: tests/test_gpu_parity.py checks next())."""
    r = torch.load(os.path.join(GOLDEN, "buffer_fake_lm.pt"), weights_only=True)
    cfg = json.loads(r["cfg"])
    buf = ca.Buffer.__new__(ca.Buffer)
    buf.cfg, buf.all_tokens = cfg, r["tokens"]
    f = [buf.estimate_norm_scaling_factor(cfg["model_batch_size"], FakeLM(r[f"{m}_table"], r[f"{m}_pos"]))
         for m in ("A", "B")]
    assert torch.equal(torch.tensor(f, dtype=torch.float32), r["normalisation_factor"])


def test_odd_shapes_keep_reference_params():
    """dict_size / d_in that are not multiples of 8: the kernels run on zero-padded dims
    (engine.padded_dims), the parameters are the reference-shaped views -- the same values as the
    reference init, a zero padding around them, and reference_state_dict() in the reference's own
    strides (the checkpoint format)."""
    cfg = _cfg("fp32", h=203, d=37)
    cc = ca.CrossCoder(cfg)
    ref = O.init_params(cfg)
    a = cc.arena()
    assert (a.h, a.d) == (208, 40) and a.padded
    for k in O.PARAM_ORDER:
        p = getattr(cc, k)
        assert p.shape == ref[k].shape and torch.equal(p.detach(), ref[k]), k
    # everything outside the views is zero
    mask = torch.ones_like(a.data, dtype=torch.bool)
    for v in a.views().values():
        v_full = torch.zeros_like(a.data, dtype=torch.bool)
        v_full.as_strided(v.shape, v.stride(), v.storage_offset())[...] = True
        mask &= ~v_full
    assert float(a.data[mask].abs().sum()) == 0.0
    sd = cc.reference_state_dict()
    for k in O.PARAM_ORDER:
        assert sd[k].stride() == ref[k].stride() and torch.equal(sd[k], ref[k]), k
    cc2 = ca.CrossCoder(dict(cfg, seed=1))
    cc2.load_state_dict(sd)
    assert all(torch.equal(getattr(cc2, k).detach(), ref[k]) for k in O.PARAM_ORDER)
