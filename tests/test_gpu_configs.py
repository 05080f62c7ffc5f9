"""BASELINE.json configs 3 / 4 / 5 at their FULL sizes on one GPU, through `Trainer.step()` (fwd + bwd +
clip + Adam on the HIP path).  The oracle cannot run these sizes in seconds, so every kernel output is
checked by size-independent properties: sampled rows / latents of each GEMM output against the
reference formulas (crosscoder.py:69-130 and their autograd) evaluated in fp64 on the GPU's own bf16
inputs of that GEMM, the loss scalars against fp64 reductions of the step's own tensors, and Adam
(torch adam.py single-tensor arithmetic, oracle.adam_update) on sampled latents against the params
before the step.  Config 3's single-GPU point has >1 GB operands (W_enc / W_dec 1.2 GB each, acts and
acts^T 1.07 GB each): the GEMMs' buffer descriptors are anchored per tile, so every offset stays far
below the 2 GB range check (gemm.hip make_rsrc / MAX_RECORDS)."""
import math

import pytest
import torch

import crosscoder_amd as ca
from oracle import cpu_reference as O

pytestmark = pytest.mark.gpu

CONFIGS = {  # BASELINE.json configs (B, n_models, d_model, dict_size)
    "config3_2x2304_131072": (4096, 2, 2304, 131072),
    "config4_2x3584_65536_b8192": (8192, 2, 3584, 65536),
    "config5_4x2304_32768": (4096, 4, 2304, 32768),
}


def rel(a, b):
    a, b = a.double(), b.double()
    return (a - b).norm().item() / max(b.norm().item(), 1e-30)


@pytest.mark.parametrize("name", list(CONFIGS))
def test_baseline_config_full_size_trainer_step(gpu, name):
    B, n, d, h = CONFIGS[name]
    K = n * d
    cfg = {"seed": 49, "batch_size": B, "buffer_mult": 128, "lr": 5e-5, "num_tokens": 400_000_000, "l1_coeff": 2,
           "beta1": 0.9, "beta2": 0.999, "dict_size": h, "seq_len": 1024, "enc_dtype": "bf16", "device": str(gpu),
           "dec_init_norm": 0.08, "d_in": d, "log_every": 100, "save_every": 30000}
    cc = ca.CrossCoder(cfg, n_models=n)
    buf = ca.SyntheticBuffer(cfg, rows=B * 2, n_models=n, seed=0)
    tr = ca.Trainer(cfg, buffer=buf, crosscoder=cc)
    tr.step_counter = 10_000  # past the l1 warm-up: l1_coeff = 2 (trainer.py:34-39)
    gi = torch.Generator().manual_seed(B + h)
    rows = torch.randint(0, B, (64,), generator=gi).to(gpu)
    lat = torch.randint(0, h, (64,), generator=gi).to(gpu)
    a = cc.arena()
    D = lambda t: t.double()  # noqa: E731  (fp64 on the GPU: the operands are too large for the host)
    We0, Wd0, be0, bd0 = (D(t).clone() for t in (a.W_enc_hk, a.W_dec_hk, a.b_enc, a.b_dec_flat))
    p_lat0 = {"W_enc": a.W_enc_hk[lat].clone(), "W_dec": a.W_dec_hk[lat].clone()}

    loss = tr.step()
    tr.synchronize()
    torch.cuda.synchronize()
    ws = cc._ws
    G = tr.optimizer.grads
    l1c = loss["l1_coeff"]
    assert l1c == 2
    x = D(ws.x)
    # G1: acts rows = relu(x W_enc^T + b_enc) (crosscoder.py:69-80)
    pre = x[rows] @ We0.t() + be0
    assert rel(D(ws.acts[rows]), pre.clamp_min(0)) < 1e-2
    flips = ((ws.acts[rows] > 0) != (pre > 0)).float().mean().item()
    assert flips <= 2e-3, flips
    # G2 (+ the loss in its epilogue): g_recon rows = bf16(2 (acts W_dec + b_dec - x) / B), crosscoder.py:82-89
    acts = D(ws.acts)
    recon = acts @ Wd0 + bd0  # fp64 reconstruction of the step's own activations
    assert rel(D(ws.g_recon[rows]), 2 * (recon[rows] - x[rows]) / B) < 8e-3
    # loss scalars vs fp64 reductions of the step's own tensors (crosscoder.py:104-128)
    l2_row = (recon - x).pow(2).sum(1)
    tn = Wd0.view(h, n, d).norm(dim=-1).sum(-1)
    assert math.isclose(loss["l2_loss"], l2_row.mean().item(), rel_tol=1e-4)
    assert math.isclose(loss["l1_loss"], (acts @ tn).mean().item(), rel_tol=1e-2)
    l0 = (ws.acts > 0).float().sum(1).mean().item()
    assert abs(loss["l0_loss"] - l0) <= 1e-6 * l0 + 1e-3  # fp32 summation order
    tv = (x - x.mean(0)).pow(2).sum(1)
    assert math.isclose(loss["explained_variance"], (1 - l2_row / (tv + 1e-8)).mean().item(), abs_tol=1e-3)
    # G3: g_pre rows = (g_recon W_dec^T + l1c tn / B) * [acts > 0]   (autograd of :84-89, :123-126)
    grec = D(ws.g_recon)
    assert rel(grec[rows], 2 * (recon[rows] - x[rows]) / B) < 1e-2
    gpre = D(ws.g_pre)
    ref3 = (grec[rows] @ Wd0.t() + l1c * tn / B) * (acts[rows] > 0)
    assert rel(gpre[rows], ref3) < 1e-2
    # G4: dW_dec latents = acts^T g_recon + l1c/B colsum(acts) W_dec/||W_dec||; G5: dW_enc = g_pre^T x
    Wd3 = Wd0.view(h, n, d)
    inv = 1.0 / Wd3.norm(dim=-1)
    l1t = (l1c / B) * acts.sum(0)[lat, None, None] * Wd3[lat] * inv[lat, :, None]
    ref4 = acts[:, lat].t() @ grec + l1t.reshape(len(lat), K)
    assert rel(D(G.W_dec_hk[lat]), ref4) < 1e-2
    assert rel(D(G.W_enc_hk[lat]), gpre[:, lat].t() @ x) < 1e-2
    assert rel(D(G.b_enc), gpre.sum(0)) < 1e-2 and rel(D(G.b_dec_flat), grec.sum(0)) < 1e-2
    # clip_grad_norm_ (trainer.py:46): the coefficient from fp64 norms of the step's own gradients
    norms = torch.stack([D(t).norm() for t in (G.W_enc_hk, G.W_dec_hk, G.b_enc, G.b_dec_flat)])
    coef = min(1.0, 1.0 / (norms.norm().item() + 1e-6))
    assert math.isclose(ws.clip_out[0].item(), coef, rel_tol=8e-3)
    # Adam (step 1, m = v = 0) on the sampled latents: oracle arithmetic in the param dtype, from the
    # params before the step and the kernel's own clip coefficient
    c = ws.clip_out[0:1].cpu()
    for k, Gk in (("W_enc", G.W_enc_hk), ("W_dec", G.W_dec_hk)):
        p = p_lat0[k].cpu()
        gk = Gk[lat].cpu() * c.to(p.dtype)
        m, v = torch.zeros_like(p), torch.zeros_like(p)
        O.adam_update(p, gk, m, v, 1.0, cfg["lr"], 0.9, 0.999, 1e-8)
        ours = getattr(a, f"{k}_hk")[lat].cpu()
        exact = (ours == p).float().mean().item()
        assert exact > 0.999, (k, exact)
        # elsewhere within one rounding of the result plus a few bf16 roundings of the update (~lr):
        # torch's bf16 intermediates (m, sqrt(v), denom) round at the update's scale
        bound = p.float().abs() * 2 ** -7 + 2 ** -5 * cfg["lr"]
        worst = ((ours.float() - p.float()).abs() / bound).max().item()
        assert worst <= 1.0, (k, worst)
    # a second step runs and the loss is finite
    loss2 = tr.step()
    assert all(math.isfinite(v) for v in loss2.values())
