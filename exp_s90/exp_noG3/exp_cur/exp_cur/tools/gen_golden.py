"""Generate golden fixtures for the crosscoder training step by running the REFERENCE
(/root/reference, read-only) on CPU in this container.

Run:  PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden.py
Out:  tests/golden/*.pt  (torch.save of plain tensors / dicts; load with weights_only=True)

The reference is imported with tools/ref_stubs.py (no LMs, no wandb).  What is exercised
is the reference's own code:
  * CrossCoder.__init__ / encode / decode / get_losses / save   (crosscoder.py:25-158)
  * Trainer.step / lr_lambda / get_l1_coeff                      (trainer.py:28-63)
    with the reference's Adam + LambdaLR + clip_grad_norm_ objects built exactly as in
    Trainer.__init__ (trainer.py:16-23); `clip_grad_norm_` is wrapped only to record the
    pre-/post-clip gradients and the returned total norm.
  * Buffer.__init__ / estimate_norm_scaling_factor / refresh / next (buffer.py) driven by a
    deterministic fake HookedTransformer (the LM forward itself is out of scope).
The fixtures are DATA (inputs + expected outputs); no reference source is copied.
This script never runs on the GPU box (it needs /root/reference).
"""
import copy
import json
import os
import shutil
import sys
import tempfile

import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "tests", "golden")


def _import_reference():
    if not os.path.isdir(REF):
        raise SystemExit("reference not present; fixtures are already committed")
    sys.dont_write_bytecode = True
    sys.path.insert(0, HERE)
    import ref_stubs

    ref_stubs.install()
    sys.path.insert(0, REF)
    import crosscoder as ref_cc  # noqa: E402
    import trainer as ref_tr  # noqa: E402
    import buffer as ref_buf  # noqa: E402

    return ref_cc, ref_tr, ref_buf


def base_cfg(B, d, h, dtype, steps):
    return {
        "seed": 49, "batch_size": B, "buffer_mult": 128, "lr": 5e-5,
        "num_tokens": B * steps, "l1_coeff": 2, "beta1": 0.9, "beta2": 0.999,
        "dict_size": h, "seq_len": 1024, "enc_dtype": dtype, "model_name": "synthetic",
        "site": "resid_pre", "device": "cpu", "model_batch_size": 4, "log_every": 100,
        "save_every": 30000, "dec_init_norm": 0.08, "hook_point": "blocks.14.hook_resid_pre",
        "wandb_project": "none", "wandb_entity": "none", "d_in": d,
    }


def synth_batch(gen, B, n, d, dtype, dyadic=False):
    """Raw activations as Buffer would hold them (enc dtype) + per-model bf16 factors."""
    if dyadic:
        raw = torch.randint(-8, 9, (B, n, d), generator=gen).float() / 8.0
        factor = torch.ones(n, dtype=torch.float32)
    else:
        raw = torch.randn(B, n, d, generator=gen)
        scales = torch.tensor([1 / 0.2759, 1 / 0.2442, 1 / 0.31, 1 / 0.27][:n])
        raw = raw * scales[None, :, None]
        # buffer.py:44-60 restated: factor = sqrt(d) / mean ||x||  (per model)
        factor = torch.tensor([(d ** 0.5) / raw[:, i].norm(dim=-1).mean().item() for i in range(n)])
    buf = raw.to(dtype)
    factor = factor.to(dtype)  # buffer.py:34-41 stores the factors in enc_dtype
    x = buf.float() * factor[None, :, None]  # buffer.py:117,124
    return buf, factor, x


def swap_nmodels(cc, n, dtype, seed):
    """n_models != 2: replace the params with n-model tensors of the same construction
    (crosscoder.py:33-62 hard-codes 2 in __init__ only)."""
    h, d = cc.W_dec.shape[0], cc.W_dec.shape[2]
    torch.manual_seed(seed)
    W_dec = torch.nn.init.normal_(torch.empty(h, n, d, dtype=dtype))
    W_dec = W_dec / W_dec.norm(dim=-1, keepdim=True) * cc.cfg["dec_init_norm"]
    cc.W_dec = torch.nn.Parameter(W_dec)
    cc.W_enc = torch.nn.Parameter(W_dec.clone().permute(1, 2, 0))  # same h-major view as :55-58
    cc.b_dec = torch.nn.Parameter(torch.zeros(n, d, dtype=dtype))


def make_dyadic_params(cc, gen):
    h, n, d = cc.W_dec.shape
    W_dec = torch.randint(-4, 5, (h, n, d), generator=gen).float() / 64.0
    with torch.no_grad():
        cc.W_dec.data = W_dec.clone()
        cc.W_enc.data = W_dec.clone().permute(1, 2, 0)
        cc.b_enc.data = (torch.randint(-4, 5, (h,), generator=gen).float() / 16.0)
        cc.b_dec.data = (torch.randint(-4, 5, (n, d), generator=gen).float() / 16.0)


class _XSource:
    def __init__(self, xs):
        self.xs = list(xs)
        self.i = 0

    def next(self):
        x = self.xs[self.i]
        self.i += 1
        return x.clone()


def build_trainer(ref_tr, cc, cfg, xs):
    """Trainer.__init__ (trainer.py:8-26) minus Buffer/wandb: same optimizer/scheduler."""
    tr = ref_tr.Trainer.__new__(ref_tr.Trainer)
    tr.cfg = cfg
    tr.crosscoder = cc
    tr.buffer = _XSource(xs)
    tr.total_steps = cfg["num_tokens"] // cfg["batch_size"]
    tr.optimizer = torch.optim.Adam(cc.parameters(), lr=cfg["lr"], betas=(cfg["beta1"], cfg["beta2"]))
    tr.scheduler = torch.optim.lr_scheduler.LambdaLR(tr.optimizer, tr.lr_lambda)
    tr.step_counter = 0
    return tr


def params_of(cc):
    return {k: v.detach().clone() for k, v in cc.state_dict().items()}


def run_case(ref_cc, ref_tr, name, B, n, d, h, dtype_s, steps, seed=0, dyadic=False, trace_fwd=True):
    dtype = ref_cc.DTYPES[dtype_s]
    cfg = base_cfg(B, d, h, dtype_s, steps)
    cc = ref_cc.CrossCoder(cfg)
    if n != 2:
        swap_nmodels(cc, n, dtype, cfg["seed"])
    gen = torch.Generator().manual_seed(1000 + seed)
    if dyadic:
        make_dyadic_params(cc, gen)
    init = params_of(cc)
    bufs, factors, xs = [], [], []
    for s in range(steps):
        b, f, x = synth_batch(gen, B, n, d, dtype, dyadic)
        bufs.append(b), factors.append(f), xs.append(x)

    rec = {"cfg": json.dumps(cfg), "n_models": n, "init": init, "buf": bufs, "factor": factors, "x": xs}

    # ---- forward trace on step-0 input (crosscoder.py:69-130) ----
    if trace_fwd:
        with torch.no_grad():
            xc = xs[0].to(dtype)
            pre = cc.encode(xc, apply_relu=False)
            acts = cc.encode(xc)
            recon = cc.decode(acts)
            fwd = cc(xc)
        lo = cc.get_losses(xs[0])
        rec["fwd"] = {
            "pre": pre, "acts": acts, "recon": recon, "forward": fwd,
            "decoder_norms": cc.W_dec.detach().norm(dim=-1),
            **{k: v.detach().clone() for k, v in lo._asdict().items()},
        }
        # backward of l2 + c*l1 for c in {0, 2}  (trainer.py:44-45)
        for c in (2.0,):  # c = 0 is step 0's pre-clip grads (rec["steps"]["clip"][0]["pre"])
            cc.zero_grad(set_to_none=True)
            lo = cc.get_losses(xs[0])
            (lo.l2_loss + c * lo.l1_loss).backward()
            rec[f"grads_l1c{int(c)}"] = {k: p.grad.detach().clone() for k, p in cc.named_parameters()}
        cc.zero_grad(set_to_none=True)

    # ---- Trainer.step sequence (trainer.py:41-63) ----
    tr = build_trainer(ref_tr, cc, cfg, xs)
    clip_log = []
    orig_clip = ref_tr.clip_grad_norm_

    def recording_clip(params, max_norm, *a, **k):
        params = list(params)
        pre = {id(p): p.grad.detach().clone() for p in params}
        tn = orig_clip(params, max_norm, *a, **k)
        names = {id(p): nm for nm, p in cc.named_parameters()}
        clip_log.append({
            "total_norm": tn.detach().clone(),
            "pre": {names[i]: g for i, g in pre.items()},
            "post": {names[id(p)]: p.grad.detach().clone() for p in params},
        })
        return tn

    ref_tr.clip_grad_norm_ = recording_clip
    try:
        dicts, after = [], {}
        keep = {0, steps - 1}
        for s in range(steps):
            dicts.append(tr.step())
            if s != 0:
                clip_log[-1] = {"total_norm": clip_log[-1]["total_norm"]}
            if s not in keep:
                continue
            st = tr.optimizer.state
            after[s] = ({
                "params": params_of(cc),
                "exp_avg": {nm: st[p]["exp_avg"].clone() for nm, p in cc.named_parameters()},
                "exp_avg_sq": {nm: st[p]["exp_avg_sq"].clone() for nm, p in cc.named_parameters()},
            })
    finally:
        ref_tr.clip_grad_norm_ = orig_clip
    rec["steps"] = {"loss_dicts": dicts, "clip": clip_log, "after": after}
    path = os.path.join(OUT, f"{name}.pt")
    torch.save(rec, path)
    print(f"{name}: {os.path.getsize(path) / 1e3:.1f} kB")


class FakeLM:
    """Deterministic stand-in for HookedTransformer.run_with_cache (buffer.py:49-53,78-86):
    activation[b, s] = table[token[b, s]] + pos[s]."""

    class _Cfg:
        pass

    def __init__(self, d, vocab, seq, seed, scale):
        g = torch.Generator().manual_seed(seed)
        self.table = torch.randn(vocab, d, generator=g) * scale
        self.pos = torch.randn(seq, d, generator=g) * scale * 0.1
        self.cfg = FakeLM._Cfg()
        self.cfg.d_model = d

    def run_with_cache(self, tokens, names_filter=None, return_type=None):
        acts = self.table[tokens] + self.pos[None, : tokens.shape[1]]
        return None, {names_filter: acts}


def run_buffer_case(ref_buf):
    """Buffer normalisation + next() protocol (buffer.py:12-125) with fake LMs."""
    d, seq, B = 16, 9, 32
    cfg = base_cfg(B, d, 64, "fp32", 4)
    cfg.update({"seq_len": seq, "buffer_mult": 4, "model_batch_size": 4})
    vocab = 50
    g = torch.Generator().manual_seed(7)
    tokens = torch.randint(0, vocab, (400, seq), generator=g)
    A, Bm = FakeLM(d, vocab, seq, 1, 3.0), FakeLM(d, vocab, seq, 2, 5.0)
    torch.manual_seed(49)
    buf = ref_buf.Buffer(cfg, A, Bm, tokens)
    rec = {"cfg": json.dumps(cfg), "tokens": tokens, "A_table": A.table, "A_pos": A.pos,
           "B_table": Bm.table, "B_pos": Bm.pos, "normalisation_factor": buf.normalisation_factor.clone(),
           "buffer_size": buf.buffer.shape[0], "next": []}
    for _ in range(6):
        rec["next"].append(buf.next().clone())
    torch.save(rec, os.path.join(OUT, "buffer_fake_lm.pt"))
    print("buffer_fake_lm:", os.path.getsize(os.path.join(OUT, "buffer_fake_lm.pt")) / 1e3, "kB")


def run_ckpt_case(ref_cc):
    cfg = base_cfg(64, 32, 256, "bf16", 1)
    tmp = tempfile.mkdtemp()
    cwd = os.getcwd()
    try:
        os.chdir(tmp)
        cc = ref_cc.CrossCoder(cfg)
        cc.save()
        cc.save()
        src = os.path.join(tmp, "checkpoints", "version_0")
        dst = os.path.join(OUT, "ckpt", "version_0")
        shutil.rmtree(dst, ignore_errors=True)
        shutil.copytree(src, dst)
    finally:
        os.chdir(cwd)
        shutil.rmtree(tmp, ignore_errors=True)
    print("ckpt: saved version_0/{0,1}.pt")


def main():
    torch.set_num_threads(1)
    os.makedirs(OUT, exist_ok=True)
    ref_cc, ref_tr, ref_buf = _import_reference()
    for dt in ("fp32", "bf16"):
        run_case(ref_cc, ref_tr, f"step_b32_n2_d32_h128_{dt}", 32, 2, 32, 128, dt, steps=10)
        run_case(ref_cc, ref_tr, f"step_b64_n2_d32_h256_{dt}", 64, 2, 32, 256, dt, steps=2)
        run_case(ref_cc, ref_tr, f"step_b96_n2_d40_h200_{dt}", 96, 2, 40, 200, dt, steps=2, seed=1)
        run_case(ref_cc, ref_tr, f"step_b64_n4_d32_h128_{dt}", 64, 4, 32, 128, dt, steps=2, seed=2)
        # d % 64 == 0: the shapes the fused G2 + loss epilogue (cc_decode_loss_t) serves in bf16
        run_case(ref_cc, ref_tr, f"step_b256_n2_d64_h512_{dt}", 256, 2, 64, 512, dt, steps=3, seed=4)
        run_case(ref_cc, ref_tr, f"step_b128_n4_d64_h256_{dt}", 128, 4, 64, 256, dt, steps=3, seed=5)
    run_case(ref_cc, ref_tr, "dyadic_b64_n2_d32_h128_fp32", 64, 2, 32, 128, "fp32", steps=1, seed=3, dyadic=True)
    run_buffer_case(ref_buf)
    run_ckpt_case(ref_cc)


if __name__ == "__main__":
    main()
