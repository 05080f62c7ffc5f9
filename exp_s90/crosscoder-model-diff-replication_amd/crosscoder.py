"""Drop-in `CrossCoder` (reference: crosscoder.py:24-217) running on gfx950 HIP kernels.

Same constructor cfg, same parameter names / shapes / dtypes / strides, same state_dict and
checkpoint format, same `encode / decode / forward / get_losses / save / load` surface.
The parameters are views of one flat HBM arena (engine.Arena) so the fused Adam can update
all of them in one launch; `W_enc` keeps the reference's h-major strides (d, 1, n*d).
"""
import json
import pprint
import weakref
from pathlib import Path
from typing import NamedTuple, Optional, Union

import torch
from torch import nn

from . import engine, ops

DTYPES = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}
SAVE_DIR = Path("./checkpoints")


class LossOutput(NamedTuple):
    l2_loss: torch.Tensor
    l1_loss: torch.Tensor
    l0_loss: torch.Tensor
    explained_variance: torch.Tensor
    explained_variance_A: torch.Tensor
    explained_variance_B: torch.Tensor


def reference_init(cfg, n_models=2):
    """Bit-exact restatement of the reference initialisation (crosscoder.py:31-62) on the CPU
    generator: seed, W_dec drawn twice (the second draw wins), per-(h, model) rows scaled to
    dec_init_norm, W_enc = rearranged clone (same values), zero biases."""
    dtype = DTYPES[cfg["enc_dtype"]]
    h, d = cfg["dict_size"], cfg["d_in"]
    torch.manual_seed(cfg["seed"])
    _ = torch.empty(n_models, d, h, dtype=dtype)  # W_enc placeholder (no RNG use)
    torch.nn.init.normal_(torch.empty(h, n_models, d, dtype=dtype))  # first draw, discarded
    W_dec = torch.nn.init.normal_(torch.empty(h, n_models, d, dtype=dtype))
    W_dec = W_dec / W_dec.norm(dim=-1, keepdim=True) * cfg["dec_init_norm"]
    return W_dec


def write_checkpoint(state_dict, cfg, save_dir=None, version=0):
    """crosscoder.py:132-146's two-file format: {save_dir}/{version}.pt (state_dict) + {version}_cfg.json,
    save_dir = ./checkpoints/version_N (next free N) when None.  Returns (save_dir, version + 1)."""
    if save_dir is None:
        SAVE_DIR.mkdir(parents=True, exist_ok=True)
        versions = [int(f.name.split("_")[1]) for f in SAVE_DIR.iterdir() if "version" in str(f)]
        save_dir = SAVE_DIR / f"version_{1 + max(versions) if versions else 0}"
        save_dir.mkdir(parents=True)
    torch.save(state_dict, save_dir / f"{version}.pt")
    with open(save_dir / f"{version}_cfg.json", "w") as f:
        json.dump(cfg, f)
    print(f"Saved as version {version} in {save_dir}")
    return save_dir, version + 1


class CrossCoder(nn.Module):
    def __init__(self, cfg, n_models: Optional[int] = None, init_W_dec: Optional[torch.Tensor] = None):
        """init_W_dec (framework extension): start from this decoder ([h, n, d], W_enc = its rearranged
        copy, zero biases) instead of the seeded reference draw -- the latent-sharded trainer passes
        its slice of the full dictionary's reference init."""
        super().__init__()
        self.cfg = cfg
        d_hidden = cfg["dict_size"]
        d_in = cfg["d_in"]
        self.n_models = int(n_models if n_models is not None else cfg.get("n_models", 2))
        self.dtype = DTYPES[cfg["enc_dtype"]]
        if self.dtype not in (torch.float32, torch.bfloat16):
            raise TypeError("crosscoder_amd kernels support enc_dtype 'bf16' and 'fp32'")
        device = torch.device(cfg["device"])
        W_dec = reference_init(cfg, self.n_models) if init_W_dec is None else init_W_dec.to(self.dtype)
        # kernel dims: dict_size / d_in rounded up to multiples of 8 (zero padding latents / columns that
        # stay zero, engine.padded_dims); the parameters are the reference-shaped views
        self._hp, self._dp = engine.padded_dims(d_hidden, d_in)
        self._arena = engine.Arena(self._hp, self.n_models, self._dp, self.dtype, device, ref=(d_hidden, d_in))
        with torch.no_grad():
            self._arena.W_dec().copy_(W_dec)
            self._arena.W_enc().copy_(W_dec.permute(1, 2, 0))
        self._bind_params()
        self.d_hidden = d_hidden
        self.save_dir = None
        self.save_version = 0
        self._ws = None

    # ------------------------------------------------------------------ arena plumbing
    def _bind_params(self):
        v = self._arena.views()
        self.W_enc = nn.Parameter(v["W_enc"])
        self.W_dec = nn.Parameter(v["W_dec"])
        self.b_enc = nn.Parameter(v["b_enc"])
        self.b_dec = nn.Parameter(v["b_dec"])

    # The Trainer runs the decoder half of Adam on a side stream (engine.adam); every public way to
    # reach the parameters orders torch's current stream after it first (a stream wait, no host sync):
    # attribute access to W_dec / b_dec, parameters() / named_parameters(), state_dict(), .to() and
    # friends (_apply), the arena re-pack, and the optimizer's state.  The step itself reaches the
    # params through the arena only, so it keeps the overlap.
    _SIDE_UPDATED = ("W_dec", "b_dec")

    def _sync_pending(self):
        a = self.__dict__.get("_arena")
        if a is not None:
            a.wait_pending()

    def __getattr__(self, name):
        if name in CrossCoder._SIDE_UPDATED:
            self._sync_pending()
        return super().__getattr__(name)

    def named_parameters(self, *args, **kwargs):
        self._sync_pending()
        return super().named_parameters(*args, **kwargs)

    def _apply(self, fn, *args, **kwargs):
        self._sync_pending()
        return super()._apply(fn, *args, **kwargs)

    def _arena_ok(self):
        a = self._arena
        v = a.views()
        for name in ("W_enc", "W_dec", "b_enc", "b_dec"):
            p = self._parameters[name]
            if p.data_ptr() != v[name].data_ptr() or p.stride() != v[name].stride() or p.device != a.data.device:
                return False
        return True

    def arena(self):
        """The flat parameter arena; re-packs the params if something (e.g. .to()) replaced them."""
        if not self._arena_ok():
            self._arena.wait_pending()  # the old arena's decoder half may still be written
            prm = self._parameters
            dev = prm["W_dec"].device
            new = engine.Arena(self._hp, self.n_models, self._dp, self.dtype, dev, ref=(self.d_hidden, self.cfg["d_in"]))
            with torch.no_grad():
                for name, dst in new.views().items():
                    dst.copy_(prm[name].data)
            self._arena = new
            grads = {n: prm[n].grad for n in ("W_enc", "W_dec", "b_enc", "b_dec")}
            self._bind_params()
            for n, g in grads.items():
                self._parameters[n].grad = g
            self._ws = None
        return self._arena

    def _workspace(self, B, step=False):
        """The cached step workspace for batch size B.  A workspace that a get_losses() graph still
        needs for its backward (ws.busy) is never reused: the next call gets a fresh one, which is
        cached in its place (so a second get_losses() before the first backward cannot overwrite
        the first one's activations)."""
        a = self.arena()
        ws = self._ws
        if (ws is None or ws.B != B or ws.x.device != a.data.device
                or (ws.busy is not None and ws.busy() is not None)):
            ws = engine.StepWorkspace(B, self.n_models, self._dp, self._hp, self.dtype, a.data.device)
            self._ws = ws
        return ws

    def _check_x(self, x):
        if x.dim() != 3 or x.shape[1] != self.n_models or x.shape[2] != self.cfg["d_in"]:
            raise ValueError(f"expected x of shape [batch, {self.n_models}, {self.cfg['d_in']}], got {tuple(x.shape)}")

    def pad_input(self, x):
        """x [batch, n, d_in] -> [batch, n, kernel d] (zero columns appended when d_in % 8 != 0)."""
        return x if self._dp == x.shape[-1] else torch.nn.functional.pad(x, (0, self._dp - x.shape[-1]))

    def _flat_x(self, x):
        self._check_x(x)
        x = self.pad_input(x).contiguous()
        if x.dtype == self.dtype:
            return x.view(x.shape[0], -1)
        return ops.prep_input(x, None, self.dtype)

    # ------------------------------------------------------------------ reference API
    def encode(self, x, apply_relu=True):
        """x [batch, n_models, d_model] -> acts [batch, d_hidden] (crosscoder.py:69-80)."""
        a = self.arena()
        xf = self._flat_x(x)
        acts = torch.empty(xf.shape[0], self._hp, dtype=self.dtype, device=xf.device)
        ops.encode_fwd(xf, a.W_enc_hk, a.b_enc, acts, apply_relu)
        return acts[:, :self.d_hidden].contiguous() if self._hp != self.d_hidden else acts

    def decode(self, acts):
        """acts [batch, d_hidden] -> [batch, n_models, d_model] incl. b_dec (crosscoder.py:82-89)."""
        a = self.arena()
        a.wait_pending()
        acts = acts.to(self.dtype)
        if self._hp != self.d_hidden:  # zero activations of the padding latents
            acts = torch.nn.functional.pad(acts, (0, self._hp - acts.shape[-1]))
        acts = acts.contiguous()
        B = acts.shape[0]
        out = torch.empty(B, self.n_models * self._dp, dtype=self.dtype, device=acts.device)
        ops.decode_fwd(acts, a.W_dec_hk, a.b_dec_flat, recon_t=out)
        out = out.view(B, self.n_models, self._dp)
        return out[:, :, :self.cfg["d_in"]].contiguous() if self._dp != self.cfg["d_in"] else out

    def forward(self, x):
        return self.decode(self.encode(x))

    def get_losses(self, x):
        """Same LossOutput as crosscoder.py:96-130; differentiable w.r.t. the four params
        (backward runs the fused HIP backward kernels)."""
        a = self.arena()
        return LossOutput(*_LossFn.apply(self, x, a.data, self.W_enc, self.W_dec, self.b_enc, self.b_dec))

    def state_dict(self, *args, **kwargs):
        # the decoder half may still be updating on the trainer's side stream
        if getattr(self, "_arena", None) is not None:
            self._arena.wait_pending()
        return super().state_dict(*args, **kwargs)

    # ------------------------------------------------------------------ checkpoints
    def create_save_dir(self):
        SAVE_DIR.mkdir(parents=True, exist_ok=True)
        versions = [int(f.name.split("_")[1]) for f in SAVE_DIR.iterdir() if "version" in str(f)]
        version = 1 + max(versions) if versions else 0
        self.save_dir = SAVE_DIR / f"version_{version}"
        self.save_dir.mkdir(parents=True)

    def save(self):
        if self.save_dir is None:
            self.create_save_dir()
        self.save_dir, self.save_version = write_checkpoint(self.reference_state_dict(), self.cfg, self.save_dir,
                                                            self.save_version)

    def reference_state_dict(self):
        """state_dict() in the reference's own tensor layout: the views themselves, or -- when the kernel
        dims are padded -- compact copies with the reference strides (W_enc [n, d, h] strides (d, 1, n*d))."""
        sd = self.state_dict()
        if not self._arena.padded:
            return sd
        out = type(sd)()
        for k, v in sd.items():
            out[k] = v.permute(2, 0, 1).contiguous().permute(1, 2, 0) if k == "W_enc" else v.contiguous()
        return out

    def _load_checked(self, state_dict):
        self.load_state_dict(state_dict)
        self.arena()

    @classmethod
    def load(cls, version_dir, checkpoint_version):
        save_dir = Path("./checkpoints") / str(version_dir)
        cfg = json.load(open(save_dir / f"{checkpoint_version}_cfg.json", "r"))
        pprint.pprint(cfg)
        self = cls(cfg=cfg)
        self._load_checked(torch.load(save_dir / f"{checkpoint_version}.pt", map_location=cfg["device"],
                                      weights_only=True))
        return self

    @classmethod
    def load_from_path(cls, cfg_path, weights_path, device: Optional[Union[str, torch.device]] = None):
        """Offline form of `load_from_hf` (crosscoder.py:160-205): a local cfg.json +
        cc_weights.pt pair (no network in this framework)."""
        with open(cfg_path, "r") as f:
            cfg = json.load(f)
        if device is not None:
            cfg["device"] = str(device)
        inst = cls(cfg)
        inst._load_checked(torch.load(weights_path, map_location=cfg["device"], weights_only=True))
        return inst

    @classmethod
    def load_from_hf(cls, repo_id="ckkissane/crosscoder-gemma-2-2b-model-diff", path="blocks.14.hook_resid_pre",
                     device=None, local_dir=None):
        """The reference downloads from the Hub; here only an already-present local copy
        ({local_dir}/{path}/cfg.json + cc_weights.pt) is read."""
        if local_dir is None:
            raise RuntimeError("load_from_hf: no network; pass local_dir with {path}/cfg.json and cc_weights.pt")
        base = Path(local_dir) / path
        return cls.load_from_path(base / "cfg.json", base / "cc_weights.pt", device)


class _GraphToken:
    """Held by one get_losses() autograd node while its backward may still run; the workspace it used
    keeps a weak reference (engine.StepWorkspace.busy)."""


class _LossFn(torch.autograd.Function):
    """get_losses as one autograd node over the fused kernels."""

    @staticmethod
    def forward(ctx, cc, x, arena_data, W_enc, W_dec, b_enc, b_dec):
        cc._check_x(x)
        ws = cc._workspace(x.shape[0])
        a = cc.arena()
        engine.forward(ws, a, cc.pad_input(x).contiguous(), None)
        s = ws.scalars
        dt = cc.dtype
        out = (s[0].clone(), s[1].to(dt, copy=True), s[2].clone(), ws.ev.clone(), ws.ev_a.to(dt, copy=True),
               ws.ev_b.to(dt, copy=True))
        ctx.cc = cc
        ctx.ws = ws
        if any(ctx.needs_input_grad[3:]):  # a graph whose backward will read ws
            ctx.token = _GraphToken()
            ws.busy = weakref.ref(ctx.token)  # freed with the graph, or cleared by backward
        ctx.mark_non_differentiable(out[2], out[3], out[4], out[5])
        return out

    @staticmethod
    def backward(ctx, g_l2, g_l1, *_):
        cc, ws = ctx.cc, ctx.ws
        a = cc.arena()
        w2 = 0.0 if g_l2 is None else float(g_l2)
        w1 = 0.0 if g_l1 is None else float(g_l1)
        if w2 != 1.0:  # g_recon was formed for d(l2)=1; re-form it for this upstream weight
            engine.loss_from_recon(ws, a, grad_scale=2.0 * w2 / ws.B)
        G = a.like()
        engine.backward(ws, a, G, l1_coeff=w1)
        ws.busy = None
        v = G.views()
        return None, None, None, v["W_enc"], v["W_dec"], v["b_enc"], v["b_dec"]
