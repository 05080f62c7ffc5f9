"""Measure how closely the fused Trainer tracks the reference's stored trajectories
(tests/golden step fixtures), to set the per-element bounds of test_trainer_steps.
For every stored step: params (max |diff| in units of lr, exact fraction, <=1 ulp fraction),
exp_avg / exp_avg_sq (relative Frobenius error), and the same statistics for a
"no Adam" stand-in (the fixture's initial params / zero moments) -- the bounds must reject it."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import crosscoder_amd as ca  # noqa: E402
from oracle import cpu_reference as O  # noqa: E402
from tests._golden import load, step_fixtures  # noqa: E402


class Replay:
    def __init__(self, bufs, factors, device):
        self.bufs = [b.to(device) for b in bufs]
        self.factors = [f.to(device) for f in factors]
        self.i = 0

    def next_raw(self):
        b, f = self.bufs[self.i], self.factors[self.i]
        self.i += 1
        return b, f


def ulp(t):
    t = t.float().abs()
    dt_bits = 7 if t.dtype == torch.bfloat16 else 23
    return torch.where(t > 0, 2.0 ** (torch.floor(torch.log2(t.clamp_min(1e-30))) - dt_bits), torch.full_like(t, 1e-30))


def pstats(p, ref, lr, dt):
    p, ref = p.float(), ref.float()
    d = (p - ref).abs()
    u = ulp(ref.to(dt)) if dt == torch.bfloat16 else ref.abs() * 2 ** -23
    return (f"max {d.max().item() / lr:7.3f} lr  exact {(d == 0).float().mean().item():.4f}  "
            f"<=1ulp {(d <= u + 1e-30).float().mean().item():.4f}  <=0.01lr {(d <= 0.01 * lr).float().mean().item():.4f}")


def rel(a, b):
    a, b = a.double(), b.double()
    return (a - b).norm().item() / max(b.norm().item(), 1e-30)


def main():
    dev = torch.device("cuda:0")
    for name in step_fixtures():
        if not name.startswith("step_"):
            continue
        r = load(name)
        cfg = dict(r["cfg"], device=str(dev))
        dt = O.DTYPES[cfg["enc_dtype"]]
        cc = ca.CrossCoder(cfg, n_models=r["n_models"])
        cc.load_state_dict(r["init"])
        tr = ca.Trainer(cfg, buffer=Replay(r["buf"], r["factor"], dev), crosscoder=cc)
        after = r["steps"]["after"]
        lr = cfg["lr"]
        print(f"== {name}")
        for s in range(len(r["x"])):
            dd = tr.step()
            ref = r["steps"]["loss_dicts"][s]
            diffs = {k: dd[k] - ref[k] for k in ref}
            print(f"  step {s} loss-dict diffs: " + ", ".join(f"{k}={v:+.3g}" for k, v in diffs.items()))
            if s not in after:
                continue
            tr.synchronize()
            st = tr.optimizer.state
            for k in O.PARAM_ORDER:
                p = getattr(cc, k).detach().cpu()
                a = after[s]
                m = st[getattr(cc, k)]["exp_avg"].cpu()
                v = st[getattr(cc, k)]["exp_avg_sq"].cpu()
                print(f"    {k:5s} ours   {pstats(p, a['params'][k], lr, dt)}  m {rel(m, a['exp_avg'][k]):.3g}"
                      f"  v {rel(v, a['exp_avg_sq'][k]):.3g}")
                print(f"    {k:5s} noAdam {pstats(r['init'][k], a['params'][k], lr, dt)}")


if __name__ == "__main__":
    main()
