"""Drop-in `Trainer` (reference: trainer.py:7-82) whose `step()` is the fused HIP step.

`step()` returns the reference's 9-key loss dict.  Per step it issues the fixed launch
sequence of engine.py and reads the 6 loss scalars once, from mapped host memory the loss-tail
kernel writes directly (the reference does 7 `.item()` syncs).  Adam state (exp_avg / exp_avg_sq, bf16 like the
reference's) lives in arenas mirroring the parameter arena, exposed through
`optimizer.state[param]` for inspection.
"""
import torch
import tqdm

from . import _hip, engine
from .buffer import Buffer
from .crosscoder import CrossCoder


def reference_loss(l2, l1, l1c, dtype):
    """The reference's logged "loss" (trainer.py:44,52): `l2_loss + l1_coeff * l1_loss` where l2 is an
    fp32 0-dim tensor and l1 one in the parameter dtype, so the product is rounded to that dtype
    first and the sum to fp32 (torch's type promotion), then `.item()`."""
    t = torch.tensor(l2, dtype=torch.float32) + l1c * torch.tensor(l1, dtype=dtype)
    return t.item()


def rounded(v, dtype):
    """float(v) rounded to the parameter dtype (the reference's param-dtype loss tensors, crosscoder.py:115-126)."""
    return float(torch.tensor(v, dtype=dtype)) if dtype != torch.float32 else float(torch.tensor(v))


class FusedAdam:
    """State holder with torch.optim.Adam's observable surface (param_groups, state)."""

    def __init__(self, cc, lr, betas, eps=1e-8):
        a = cc.arena()
        self.cc = cc
        self.exp_avg = a.like()
        self.exp_avg_sq = a.like()
        self.grads = a.like()
        self.param_groups = [{"lr": lr, "initial_lr": lr, "betas": betas, "eps": eps, "weight_decay": 0.0}]
        self.t = 0

    @property
    def state(self):
        self.cc.arena().wait_pending()  # the decoder half may still be updating on the side stream
        m, v = self.exp_avg.views(), self.exp_avg_sq.views()
        st = {}
        for name in ("W_enc", "W_dec", "b_enc", "b_dec"):
            p = getattr(self.cc, name)
            st[p] = {"step": torch.tensor(float(self.t)), "exp_avg": m[name], "exp_avg_sq": v[name]}
        return st

    def zero_grad(self, set_to_none=True):
        pass  # grads are overwritten (never accumulated) by the backward kernels


class LambdaLRHost:
    """torch.optim.lr_scheduler.LambdaLR over one group, evaluated on the host."""

    def __init__(self, optimizer, lr_lambda):
        self.optimizer = optimizer
        self.lr_lambda = lr_lambda
        self.base_lr = optimizer.param_groups[0]["initial_lr"]
        self.last_epoch = 0
        optimizer.param_groups[0]["lr"] = self.base_lr * lr_lambda(0)
        self._last_lr = [optimizer.param_groups[0]["lr"]]

    def step(self):
        self.last_epoch += 1
        lr = self.base_lr * self.lr_lambda(self.last_epoch)
        self.optimizer.param_groups[0]["lr"] = lr
        self._last_lr = [lr]

    def get_last_lr(self):
        return list(self._last_lr)


class Trainer:
    def __init__(self, cfg, model_A=None, model_B=None, all_tokens=None, buffer=None, crosscoder=None, logger=None):
        self.cfg = cfg
        self.model_A = model_A
        self.model_B = model_B
        self.crosscoder = crosscoder if crosscoder is not None else CrossCoder(cfg)
        self.buffer = buffer if buffer is not None else Buffer(cfg, model_A, model_B, all_tokens)
        self.total_steps = cfg["num_tokens"] // cfg["batch_size"]
        self.optimizer = FusedAdam(self.crosscoder, cfg["lr"], (cfg["beta1"], cfg["beta2"]))
        self.scheduler = LambdaLRHost(self.optimizer, self.lr_lambda)
        self.step_counter = 0
        self.logger = logger
        self._mapped = None  # mapped host words the step's loss tail writes (allocated on the first step)
        self._seq = 0
        self._side = None  # stream of the decoder half's Adam (created on the first step)
        self._last_ws = None  # the last step's workspace (its G2 abort word, engine.check_step_abort)

    def lr_lambda(self, step):
        if step < 0.8 * self.total_steps:
            return 1.0
        return 1.0 - (step - 0.8 * self.total_steps) / (0.2 * self.total_steps)

    def get_l1_coeff(self):
        if self.step_counter < 0.05 * self.total_steps:
            return self.cfg["l1_coeff"] * self.step_counter / (0.05 * self.total_steps)
        return self.cfg["l1_coeff"]

    def _launch_step(self, host, seq):
        """The step's launches; the loss tail writes the scalars to `host` (a _hip.MappedHostBuffer), then `seq`:
        the host waits for that word, not for a stream.  Only step() launches a step, and it checks the step's abort
        word before the next one is launched (_check_abort): a timed-out G2 aborts exactly one step, whose rollback
        of the optimizer's step count and LR schedule happens in that same step()."""
        cc = self.crosscoder
        raw, factor = self.buffer.next_raw()
        raw = cc.pad_input(raw)  # (zero columns only when d_in % 8 != 0)
        ws = cc._workspace(raw.shape[0], step=True)
        P = cc.arena()
        opt = self.optimizer
        side = self._side_stream()
        # prep, G1, G2 + the loss rows (one pass where decode_loss_t serves the shape)
        engine.forward(ws, P, raw, factor if getattr(self.buffer, "normalize", True) else None, finalize=False)
        # the loss scalars: into mapped host memory from the G3 launch (or, where G3 cannot carry the tail, from a
        # launch on the side stream beside G3)
        engine.loss_finalize_with_g3(ws, side, host=host, seq=seq)
        l1c = self.get_l1_coeff()
        # clip_grad_norm_(max_norm=1.0), trainer.py:46
        engine.backward(ws, P, opt.grads, l1c, clip=1.0)
        g = opt.param_groups[0]
        opt.t += 1
        b1, b2 = g["betas"]
        engine.clip_and_adam(ws, P, opt.grads, opt.exp_avg, opt.exp_avg_sq, g["lr"], b1, b2, g["eps"], opt.t,
                             side_stream=side)
        self.scheduler.step()
        self._last_l1c = l1c
        self._last_ws = ws

    def _side_stream(self):
        # the decoder half of Adam (+ the next step's decoder norms / W_dec^T) runs here, beside the
        # next step's prep / encoder GEMM (engine.adam)
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.crosscoder.arena().data.device)
        return self._side

    def synchronize(self):
        """Order torch's current stream after every launch of the last step (the decoder half of
        Adam may still run on the side stream, and its last rows are deferred to the next reader, which
        launches them; CrossCoder's accessors and optimizer.state do this by themselves)."""
        self.crosscoder.arena().wait_pending()
        self._check_abort()

    def _check_abort(self):
        """Raise engine.STEP_ABORTED_MSG if the last step's G2 timed out waiting for the side-stream Adam; its
        launches applied no update, so the optimizer's step count and the LR schedule are rolled back."""
        try:
            engine.check_step_abort(self._last_ws)
        except RuntimeError:
            self.optimizer.t -= 1
            self.scheduler.last_epoch -= 1
            lr = self.scheduler.base_lr * self.lr_lambda(self.scheduler.last_epoch)
            self.optimizer.param_groups[0]["lr"] = lr
            self.scheduler._last_lr = [lr]
            raise

    def step(self):
        if self._mapped is None:
            self._mapped = _hip.MappedHostBuffer(16)
        self._seq = (self._seq + 1) & 0xFFFFFFFF or 1
        self._launch_step(self._mapped, self._seq)
        self._mapped.wait(8, self._seq)
        self._check_abort()  # (G2 timed out: raise in THIS step; its Adam launches applied nothing)
        s = [float(v) for v in self._mapped.f32[:6]]
        l1c = self._last_l1c
        dt = self.crosscoder.dtype
        l2, l1, l0 = s[0], rounded(s[1], dt), s[2]
        loss_dict = {
            "loss": reference_loss(l2, l1, l1c, dt),
            "l2_loss": l2,
            "l1_loss": l1,
            "l0_loss": l0,
            "l1_coeff": l1c,
            "lr": self.scheduler.get_last_lr()[0],
            "explained_variance": s[3],
            "explained_variance_A": rounded(s[4], dt),
            "explained_variance_B": rounded(s[5], dt),
        }
        self.step_counter += 1
        return loss_dict

    def log(self, loss_dict):
        if self.logger is not None:
            self.logger(loss_dict, self.step_counter)
        print(loss_dict)

    def save(self):
        self.synchronize()
        self.crosscoder.save()

    def train(self):
        self.step_counter = 0
        try:
            for i in tqdm.trange(self.total_steps):
                loss_dict = self.step()
                if i % self.cfg["log_every"] == 0:
                    self.log(loss_dict)
                if (i + 1) % self.cfg["save_every"] == 0:
                    self.save()
        finally:
            self.save()
