"""Weight-space utilities around the crosscoder, on the GPU kernels:

* `decoder_stats(cc)` -- the decoder-norm analysis of analysis.py:9-40 (per-latent norms per
  model, relative decoder norm strength, the shared-latent mask, cosine similarity of the two
  models' decoder vectors) in one HBM pass over W_dec (cc_decoder_stats).
* `fold_activation_scaling_factor(cc, *scales)` -- Crosscoder_model_diff.ipynb:35368-35378: fold the
  per-model activation normalisation factors into the weights (W_enc[m] *= s_m, W_dec[:, m] /= s_m,
  b_dec[m] /= s_m) so the crosscoder takes raw residual-stream activations (cc_fold_scaling).
* `sae_vis_export(cc, *scales)` -- the notebook's latent-dashboard hand-off (:35735-35801): a copy with
  the scaling factors folded into W_enc only, whose state_dict the sae_vis fork's CrossCoder loads
  (`load_state_dict(folded_cross_coder.state_dict())`, keys / shapes of the reference), plus the
  CrossCoderConfig fields that fork is built with.
"""
import torch

from . import ops


def decoder_stats(cc, shared_range=(0.3, 0.7)):
    """analysis.py:9-12 (norms, relative_norms = norms[:, 1] / norms.sum(-1)), :35 (shared-latent mask
    0.3 < rel < 0.7), :40 (cosine_sims).  fp32 results on the crosscoder's device."""
    a = cc.arena()
    a.wait_pending()
    norms, rel, cos = ops.decoder_stats(a.W_dec_hk, a.n, a.d)
    if a.padded:  # (the padding columns are zero: the padding latents are dropped)
        norms, rel, cos = norms[:a.h_ref], rel[:a.h_ref], cos[:a.h_ref]
    lo, hi = shared_range
    return {"norms": norms, "relative_norms": rel, "shared_latent_mask": (rel < hi) & (rel > lo),
            "cosine_sims": cos}


def fold_activation_scaling_factor(cross_coder, *scaling_factors, fold_decoder=True):
    """In place, returns the crosscoder (the notebook's two-model signature:
    fold_activation_scaling_factor(cc, base_scaling_factor, chat_scaling_factor)).
    fold_decoder=False folds the encoder only (the notebook's second variant, :35752-35763)."""
    a = cross_coder.arena()
    a.wait_pending()
    if len(scaling_factors) != a.n:
        raise ValueError(f"expected {a.n} scaling factors, got {len(scaling_factors)}")
    s = torch.tensor([float(f) for f in scaling_factors], dtype=torch.float32, device=a.data.device)
    # the encoder-only variant passes no decoder pointers
    ops.fold_scaling(a.W_enc_hk, a.W_dec_hk if fold_decoder else None, a.b_dec_flat if fold_decoder else None, s,
                     a.n, a.d)
    return cross_coder


def sae_vis_export(cross_coder, *scaling_factors, dtype=torch.bfloat16):
    """-> (state_dict on the CPU in `dtype`, sae_vis CrossCoderConfig kwargs).  The crosscoder itself
    is left untouched (the notebook folds a deep copy, :35752-35763)."""
    import copy

    a = cross_coder.arena()
    a.wait_pending()
    ws, cross_coder._ws = cross_coder._ws, None  # (no copy of the step workspace)
    try:
        folded = copy.deepcopy(cross_coder)
    finally:
        cross_coder._ws = ws
    fold_activation_scaling_factor(folded, *scaling_factors, fold_decoder=False)
    sd = {k: v.detach().to("cpu", dtype) for k, v in folded.reference_state_dict().items()}
    cfg = {"d_in": cross_coder.cfg["d_in"], "d_hidden": cross_coder.cfg["dict_size"], "apply_b_dec_to_input": False}
    return sd, cfg
