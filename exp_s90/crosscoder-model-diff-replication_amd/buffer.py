"""Activation buffers feeding the step (reference: buffer.py:8-125).

`Buffer` keeps the reference's constructor and `next()` contract: it harvests activations
from two (or more) models through their `run_with_cache` hook API, estimates the per-model
norm-scaling factors (sqrt(d_model) / mean ||x||, buffer.py:44-63), keeps the buffer in HBM
in enc_dtype, shuffles it on refresh and hands out batches.  The LM forward itself is the
caller's model (out of scope for the kernels); the shuffle is a GPU row gather (cc_gather_rows),
so the buffer lives on a ROCm device.  `next_raw()` is the zero-copy form used by
the fused Trainer: a [batch, n, d] slice of the HBM buffer plus the factors, which the
prologue kernel (cc_prep_input) scales and casts in one pass.

`SyntheticBuffer` is the same protocol over seeded synthetic activations (no LMs) — the
benchmark's data source.
"""
import numpy as np
import torch
import tqdm

from . import ops
from .crosscoder import DTYPES



class _BufferProtocol:
    normalize = True

    def next(self):
        """fp32 [batch, n, d], scaled by the normalisation factors (buffer.py:115-125)."""
        raw, factor = self.next_raw()
        out = raw.float()
        if self.normalize:
            out = out * factor[None, :, None]
        return out


class Buffer(_BufferProtocol):
    def __init__(self, cfg, model_A, model_B, all_tokens, models=None):
        self.models = list(models) if models is not None else [model_A, model_B]
        d = self.models[0].cfg.d_model
        assert all(m.cfg.d_model == d for m in self.models)
        self.cfg = cfg
        self.n = len(self.models)
        self.buffer_size = cfg["batch_size"] * cfg["buffer_mult"]
        self.buffer_batches = self.buffer_size // (cfg["seq_len"] - 1)
        self.buffer_size = self.buffer_batches * (cfg["seq_len"] - 1)
        self.dtype = DTYPES[cfg["enc_dtype"]]
        self.buffer = torch.zeros((self.buffer_size, self.n, d), dtype=self.dtype, device=cfg["device"])
        self.token_pointer = 0
        self.first = True
        self.normalize = True
        self.all_tokens = all_tokens
        self._spare = None
        factors = [self.estimate_norm_scaling_factor(cfg["model_batch_size"], m) for m in self.models]
        self.normalisation_factor = torch.tensor(factors, device=cfg["device"], dtype=self.dtype)
        self.refresh()

    @torch.no_grad()
    def estimate_norm_scaling_factor(self, batch_size, model, n_batches_for_norm_estimate: int = 100):
        norms = []
        for i in tqdm.tqdm(range(n_batches_for_norm_estimate), desc="Estimating norm scaling factor"):
            tokens = self.all_tokens[i * batch_size: (i + 1) * batch_size]
            _, cache = model.run_with_cache(tokens, names_filter=self.cfg["hook_point"], return_type=None)
            norms.append(cache[self.cfg["hook_point"]].norm(dim=-1).mean().item())
        return np.sqrt(model.cfg.d_model) / np.mean(norms)

    @torch.no_grad()
    def refresh(self):
        self.buffer_pointer = 0
        num_batches = self.buffer_batches if self.first else self.buffer_batches // 2
        self.first = False
        mbs = self.cfg["model_batch_size"]
        hp = self.cfg["hook_point"]
        for b0 in tqdm.trange(0, num_batches, mbs):
            tokens = self.all_tokens[self.token_pointer + b0: self.token_pointer + min(b0 + mbs, num_batches)]
            caches = [m.run_with_cache(tokens, names_filter=hp)[1][hp] for m in self.models]
            acts = torch.stack(caches, dim=0)[:, :, 1:, :]  # drop BOS
            assert acts.shape == (self.n, tokens.shape[0], tokens.shape[1] - 1, self.buffer.shape[-1])
            acts = acts.permute(1, 2, 0, 3).reshape(-1, self.n, self.buffer.shape[-1])
            self.buffer[self.buffer_pointer: self.buffer_pointer + acts.shape[0]] = acts
            self.buffer_pointer += acts.shape[0]
        self.token_pointer += num_batches
        self.buffer_pointer = 0
        # buffer = buffer[randperm(rows)] (buffer.py:111-113): the permutation from torch's global CPU
        # generator exactly as the reference draws it, the row gather on the GPU (cc_gather_rows)
        # into a second resident buffer; the two buffers swap roles every refresh
        perm = torch.randperm(self.buffer.shape[0]).to(self.buffer.device)
        spare = self._spare
        if spare is None or spare.shape != self.buffer.shape or spare.dtype != self.buffer.dtype:
            spare = torch.empty_like(self.buffer)
        ops.gather_rows(self.buffer, perm, out=spare)
        self._spare, self.buffer = self.buffer, spare

    def next_raw(self):
        B = self.cfg["batch_size"]
        out = self.buffer[self.buffer_pointer: self.buffer_pointer + B]
        self.buffer_pointer += B
        if self.buffer_pointer > self.buffer.shape[0] // 2 - B:
            # refresh overwrites the first half of the buffer in place.  The reference's
            # `.float()` (buffer.py:117) copies only when enc_dtype is not fp32; for fp32 it
            # aliases and the returned batch sees the overwrite -- kept for identical batches.
            if out.dtype != torch.float32:
                out = out.clone()
            self.refresh()
        return out, self.normalisation_factor


class SyntheticBuffer(_BufferProtocol):
    """Seeded synthetic residual-stream stand-in: x ~ N(0,1) per model scaled by 1/factor
    (Gemma-2-2b base/IT scale factors, Crosscoder_model_diff.ipynb:35379-35380), stored in
    HBM in enc_dtype; factors estimated with the reference's formula."""

    RAW_SCALES = (1 / 0.2759, 1 / 0.2442, 1 / 0.31, 1 / 0.27)

    def __init__(self, cfg, rows, n_models=2, seed=0, device=None):
        device = device or cfg["device"]
        self.cfg = cfg
        self.dtype = DTYPES[cfg["enc_dtype"]]
        d = cfg["d_in"]
        g = torch.Generator(device=device).manual_seed(seed)
        scales = torch.tensor([self.RAW_SCALES[i % 4] for i in range(n_models)], device=device)
        buf = torch.empty(rows, n_models, d, dtype=self.dtype, device=device)
        chunk = 65536
        for r0 in range(0, rows, chunk):
            r1 = min(rows, r0 + chunk)
            z = torch.randn(r1 - r0, n_models, d, generator=g, device=device)
            buf[r0:r1] = (z * scales[None, :, None]).to(self.dtype)
        self.buffer = buf
        sample = buf[: min(rows, 4096)].float()
        f = [(d ** 0.5) / sample[:, i].norm(dim=-1).mean().item() for i in range(n_models)]
        self.normalisation_factor = torch.tensor(f, device=device, dtype=self.dtype)
        self.buffer_pointer = 0

    def next_raw(self):
        B = self.cfg["batch_size"]
        if self.buffer_pointer + B > self.buffer.shape[0]:
            self.buffer_pointer = 0
        out = self.buffer[self.buffer_pointer: self.buffer_pointer + B]
        self.buffer_pointer += B
        return out, self.normalisation_factor
