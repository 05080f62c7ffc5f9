"""ORACLE — test infrastructure only, never shipped or measured as the product.

CPU restatement (pure torch, same op sequence as the reference so that CPU results are
bit-identical) of the crosscoder training step of mitroitskii/crosscoder-model-diff-replication.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this file.

Pinned against golden fixtures produced by running the reference itself on CPU
(tools/gen_golden.py -> tests/golden/*.pt; tests/test_oracle_golden.py checks bit-equality).

Restated reference code:
  init        crosscoder.py:31-62     encode   crosscoder.py:69-80
  decode      crosscoder.py:82-89     losses   crosscoder.py:96-130
  step        trainer.py:41-63        lr_lambda / get_l1_coeff trainer.py:28-39
  clip        torch/nn/utils/clip_grad.py (_get_total_norm, _clip_grads_with_norm_)
  Adam        torch/optim/adam.py:_single_tensor_adam (no weight decay, no amsgrad)
  Buffer.next buffer.py:115-125
"""
import einops
import torch

DTYPES = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}
PARAM_ORDER = ("W_enc", "W_dec", "b_enc", "b_dec")


def init_params(cfg, n_models=2):
    """crosscoder.py:31-62 (double normal_ draw, row-normalised, W_enc = permuted clone)."""
    dtype = DTYPES[cfg["enc_dtype"]]
    h, d = cfg["dict_size"], cfg["d_in"]
    torch.manual_seed(cfg["seed"])
    torch.nn.init.normal_(torch.empty(h, n_models, d, dtype=dtype))
    W_dec = torch.nn.init.normal_(torch.empty(h, n_models, d, dtype=dtype))
    W_dec = W_dec / W_dec.norm(dim=-1, keepdim=True) * cfg["dec_init_norm"]
    W_enc = W_dec.clone().permute(1, 2, 0)
    return {
        "W_enc": W_enc, "W_dec": W_dec,
        "b_enc": torch.zeros(h, dtype=dtype), "b_dec": torch.zeros(n_models, d, dtype=dtype),
    }


def encode(x, P, apply_relu=True):
    """crosscoder.py:69-80."""
    pre = einops.einsum(x, P["W_enc"], "batch n_models d_model, n_models d_model d_hidden -> batch d_hidden")
    return torch.relu(pre + P["b_enc"]) if apply_relu else pre + P["b_enc"]


def decode(acts, P):
    """crosscoder.py:82-89."""
    r = einops.einsum(acts, P["W_dec"], "batch d_hidden, d_hidden n_models d_model -> batch n_models d_model")
    return r + P["b_dec"]


def get_losses(x, P, dtype):
    """crosscoder.py:96-130; returns a dict with the LossOutput fields."""
    x = x.to(dtype)
    acts = encode(x, P)
    recon = decode(acts, P)
    diff = recon.float() - x.float()
    l2_per_batch = diff.pow(2).sum(dim=(1, 2))
    l2_loss = l2_per_batch.mean()
    eps = 1e-8
    total_variance = (x - x.mean(0)).pow(2).sum(dim=(1, 2))
    ev = 1 - l2_per_batch / (total_variance + eps)
    ev_m = []
    for m in (0, 1):
        per_tok = (recon[:, m, :] - x[:, m, :]).pow(2).sum(dim=-1).squeeze()
        tv = (x[:, m, :] - x[:, m, :].mean(0)).pow(2).sum(-1).squeeze()
        ev_m.append(1 - per_tok / (tv + eps))
    decoder_norms = P["W_dec"].norm(dim=-1)
    total_decoder_norm = decoder_norms.sum(dim=1)
    l1_loss = (acts * total_decoder_norm[None, :]).sum(-1).mean(0)
    l0_loss = (acts > 0).float().sum(-1).mean()
    return {"l2_loss": l2_loss, "l1_loss": l1_loss, "l0_loss": l0_loss, "explained_variance": ev,
            "explained_variance_A": ev_m[0], "explained_variance_B": ev_m[1]}


def lr_lambda(step, total_steps):
    """trainer.py:28-32."""
    if step < 0.8 * total_steps:
        return 1.0
    return 1.0 - (step - 0.8 * total_steps) / (0.2 * total_steps)


def l1_coeff(step_counter, total_steps, l1):
    """trainer.py:34-39."""
    if step_counter < 0.05 * total_steps:
        return l1 * step_counter / (0.05 * total_steps)
    return l1


def clip_grad_norm(grads, max_norm=1.0):
    """clip_grad_norm_: per-tensor 2-norms -> norm of the stacked norms -> scale in place."""
    norms = [torch.linalg.vector_norm(g, 2.0) for g in grads]
    total = torch.linalg.vector_norm(torch.stack(norms), 2.0)
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    for g in grads:
        g.mul_(coef)
    return total


def adam_update(p, g, m, v, step, lr, beta1, beta2, eps):
    """torch.optim.Adam single-tensor update (adam.py), step = count after increment."""
    m.lerp_(g, 1 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    step_size = lr / bc1
    denom = (v.sqrt() / (bc2 ** 0.5)).add_(eps)
    p.addcdiv_(m, denom, value=-step_size)


def loss_and_grads(x, P, dtype, l1c):
    """autograd of l2 + l1c * l1 (trainer.py:44-45) on leaf copies of P."""
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in P.items()}  # clone keeps strides
    lo = get_losses(x, leaves, dtype)
    loss = lo["l2_loss"] + l1c * lo["l1_loss"]
    loss.backward()
    return lo, loss, {k: leaves[k].grad for k in PARAM_ORDER}


class OracleTrainer:
    """Trainer.step (trainer.py:41-63) restated over a dict of CPU tensors."""

    def __init__(self, cfg, P, n_models=2):
        self.cfg = cfg
        self.dtype = DTYPES[cfg["enc_dtype"]]
        self.P = {k: torch.nn.Parameter(v.detach().clone()) for k, v in P.items()}  # clone keeps strides
        self.total_steps = cfg["num_tokens"] // cfg["batch_size"]
        self.step_counter = 0
        self.m = {k: torch.zeros_like(v) for k, v in self.P.items()}
        self.v = {k: torch.zeros_like(v) for k, v in self.P.items()}
        self.t = 0
        self.lr = cfg["lr"] * lr_lambda(0, self.total_steps)
        self.last_total_norm = None

    def step(self, x):
        l1c = l1_coeff(self.step_counter, self.total_steps, self.cfg["l1_coeff"])
        lo = get_losses(x, self.P, self.dtype)
        loss = lo["l2_loss"] + l1c * lo["l1_loss"]
        for p in self.P.values():
            p.grad = None
        loss.backward()
        params = [self.P[k] for k in PARAM_ORDER]
        with torch.no_grad():
            self.last_total_norm = clip_grad_norm([p.grad for p in params])
            self.t += 1
            for k in PARAM_ORDER:
                adam_update(self.P[k].data, self.P[k].grad, self.m[k], self.v[k], float(self.t), self.lr,
                            self.cfg["beta1"], self.cfg["beta2"], 1e-8)
        self.lr = self.cfg["lr"] * lr_lambda(self.t, self.total_steps)
        d = {
            "loss": loss.item(), "l2_loss": lo["l2_loss"].item(), "l1_loss": lo["l1_loss"].item(),
            "l0_loss": lo["l0_loss"].item(), "l1_coeff": l1c, "lr": self.lr,
            "explained_variance": lo["explained_variance"].mean().item(),
            "explained_variance_A": lo["explained_variance_A"].mean().item(),
            "explained_variance_B": lo["explained_variance_B"].mean().item(),
        }
        self.step_counter += 1
        return d


def buffer_next(buf_rows, factor):
    """buffer.py:117,124: slice.float() * factor[None, :, None]."""
    return buf_rows.float() * factor[None, :, None]


def step_flops(B, n, d, h):
    """Algorithmic work of one step: 5 GEMMs x 2*B*(n*d)*h."""
    return 10.0 * B * n * d * h


def isclose_rel(a, b):
    a, b = a.double(), b.double()
    return (a - b).norm().item() / max(b.norm().item(), 1e-30)

