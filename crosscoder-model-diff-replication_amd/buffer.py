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

Latent-sharded training (sharded.py) needs every rank to train on the SAME rows ("replicate x").
`Buffer(..., group=g)` makes that hold by construction instead of by identical RNG state and LM outputs: each
rank harvests a contiguous 1/G of every refresh's LM batches (and of the norm-estimate batches) and the others
receive them by broadcast, and the shuffle's permutation is drawn on the group's rank 0 -- from torch's global
CPU generator, as the reference does -- and broadcast.  Rank 0 of a group therefore holds exactly the buffer a
single-process `Buffer` would, and every other rank a copy of it.  `fingerprint()` (a position-weighted integer
checksum of the buffer and the factors) is what `ShardedTrainer` compares across ranks after every refresh.
"""
import numpy as np
import torch
import torch.distributed as dist
import tqdm

from . import ops
from .crosscoder import DTYPES



def _coll_device(group, default):
    """Where the group's collectives take their tensors: the GPU for RCCL ("nccl"), else `default`."""
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return default


def _src(group, r):
    """Global rank of the group's rank r (broadcast's src)."""
    return dist.get_global_rank(group, r) if group is not None and group != dist.group.WORLD else r


def fingerprint(buf, factor):
    """int64 [2]: a position-weighted checksum of the buffer's bits (sum over rows of (row % 4093 + 1) times the
    row's sum of 16-bit words; |partial sums| < 2^60 for buffers up to 2^19 rows of 9216 words) and of the
    normalisation factors' bits.  Equal on two ranks <=> (almost surely) the same rows in the same order."""
    words = buf.reshape(buf.shape[0], -1).view(torch.int16)
    rows = words.shape[0]
    total = torch.zeros((), dtype=torch.int64, device=buf.device)
    step = 4096
    for r0 in range(0, rows, step):
        r1 = min(rows, r0 + step)
        w = (torch.arange(r0, r1, device=buf.device, dtype=torch.int64) % 4093) + 1
        total += (words[r0:r1].sum(dim=1, dtype=torch.int64) * w).sum()
    f = factor.reshape(-1).contiguous().view(torch.int16).to(torch.int64)
    fw = (torch.arange(f.numel(), device=f.device, dtype=torch.int64) + 1) * f
    return torch.stack([total, fw.sum().to(total.device)])


class _BufferProtocol:
    normalize = True
    refresh_count = 0  # refreshes so far (ShardedTrainer re-checks the ranks' fingerprints when it changes)

    def fingerprint(self):
        return fingerprint(self.buffer, self.normalisation_factor)

    def next(self):
        """fp32 [batch, n, d], scaled by the normalisation factors (buffer.py:115-125)."""
        raw, factor = self.next_raw()
        out = raw.float()
        if self.normalize:
            out = out * factor[None, :, None]
        return out


class Buffer(_BufferProtocol):
    # the refresh's row gather (cc_gather_rows; the tests of the group logic on CPU substitute torch indexing)
    gather_rows = staticmethod(ops.gather_rows)

    def __init__(self, cfg, model_A, model_B, all_tokens, models=None, group=None):
        """group: a torch.distributed process group whose ranks share this buffer (the latent-sharded step): the
        harvest is split over them and the results broadcast, the shuffle drawn on its rank 0 (module doc).
        None: the reference's single-process buffer."""
        self.group = group
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

    def _share(self, n):
        """[lo, hi) of the n items (LM batches) this rank harvests: a contiguous 1/G of them; all n alone."""
        group = getattr(self, "group", None)
        if group is None:
            return 0, n
        G, r = dist.get_world_size(group), dist.get_rank(group)
        return r * n // G, (r + 1) * n // G

    @torch.no_grad()
    def estimate_norm_scaling_factor(self, batch_size, model, n_batches_for_norm_estimate: int = 100):
        lo, hi = self._share(n_batches_for_norm_estimate)
        norms = [0.0] * n_batches_for_norm_estimate
        for i in tqdm.tqdm(range(lo, hi), desc="Estimating norm scaling factor"):
            tokens = self.all_tokens[i * batch_size: (i + 1) * batch_size]
            _, cache = model.run_with_cache(tokens, names_filter=self.cfg["hook_point"], return_type=None)
            norms[i] = cache[self.cfg["hook_point"]].norm(dim=-1).mean().item()
        group = getattr(self, "group", None)
        if group is not None:
            # every rank's batches into one list (each entry is one rank's float64 value plus zeros: exact), in
            # batch order, so the mean below is the single-process one bit for bit
            t = torch.tensor(norms, dtype=torch.float64, device=_coll_device(group, "cpu"))
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
            norms = t.cpu().tolist()
        return np.sqrt(model.cfg.d_model) / np.mean(norms)

    @torch.no_grad()
    def refresh(self):
        self.buffer_pointer = 0
        num_batches = self.buffer_batches if self.first else self.buffer_batches // 2
        self.first = False
        mbs = self.cfg["model_batch_size"]
        hp = self.cfg["hook_point"]
        seq_rows = self.all_tokens.shape[1] - 1  # rows per sequence (BOS dropped)
        starts = list(range(0, num_batches, mbs))
        lo, hi = self._share(len(starts))  # (all of them without a group)
        for c in tqdm.trange(lo, hi):
            b0 = starts[c]
            tokens = self.all_tokens[self.token_pointer + b0: self.token_pointer + min(b0 + mbs, num_batches)]
            caches = [m.run_with_cache(tokens, names_filter=hp)[1][hp] for m in self.models]
            acts = torch.stack(caches, dim=0)[:, :, 1:, :]  # drop BOS
            assert acts.shape == (self.n, tokens.shape[0], tokens.shape[1] - 1, self.buffer.shape[-1])
            acts = acts.permute(1, 2, 0, 3).reshape(-1, self.n, self.buffer.shape[-1])
            r0 = b0 * seq_rows  # (= the reference's running buffer_pointer)
            self.buffer[r0: r0 + acts.shape[0]] = acts
        group = getattr(self, "group", None)
        if group is not None:
            # rank r's contiguous rows to every other rank
            G = dist.get_world_size(group)
            for r in range(G):
                c0, c1 = r * len(starts) // G, (r + 1) * len(starts) // G
                if c0 == c1:
                    continue
                r0, r1 = starts[c0] * seq_rows, min(num_batches, starts[c1 - 1] + mbs) * seq_rows
                dist.broadcast(self.buffer[r0:r1], src=_src(group, r), group=group)
        self.token_pointer += num_batches
        self.buffer_pointer = 0
        # buffer = buffer[randperm(rows)] (buffer.py:111-113): the permutation from torch's global CPU
        # generator exactly as the reference draws it (on the group's rank 0, then broadcast), the row gather on
        # the GPU (cc_gather_rows) into a second resident buffer; the two buffers swap roles every refresh
        rows = self.buffer.shape[0]
        if group is None:
            perm = torch.randperm(rows).to(self.buffer.device)
        else:
            perm = torch.randperm(rows) if dist.get_rank(group) == 0 else torch.empty(rows, dtype=torch.int64)
            perm = perm.to(_coll_device(group, self.buffer.device))
            dist.broadcast(perm, src=_src(group, 0), group=group)
            perm = perm.to(self.buffer.device)
        spare = self._spare
        if spare is None or spare.shape != self.buffer.shape or spare.dtype != self.buffer.dtype:
            spare = torch.empty_like(self.buffer)
        self.gather_rows(self.buffer, perm, out=spare)
        self._spare, self.buffer = self.buffer, spare
        self.refresh_count += 1

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
