"""Stub modules that let the read-only reference (/root/reference) be imported on CPU
in THIS container, for golden-fixture generation only.

The reference's `utils.py` imports IPython, transformer_lens, jaxtyping and wandb at
module scope (utils.py:3,26-28,32,34,41; buffer.py:2); none of them is on the
arithmetic path of `CrossCoder.get_losses` / `Trainer.step`.  This file never ships to
the GPU box as a dependency of the product and is not imported by the package.
"""
import sys
import types


def _mod(name, **attrs):
    m = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


class _Dummy:
    def __init__(self, *a, **k):
        pass

    def __call__(self, *a, **k):
        return None

    def __getattr__(self, item):
        return _Dummy()


def install():
    _mod("IPython", get_ipython=lambda: None)
    _mod("IPython.display", HTML=_Dummy)
    tl = _mod("transformer_lens", HookedTransformer=_Dummy, ActivationCache=dict)
    tl.hook_points = _mod("transformer_lens.hook_points", HookPoint=_Dummy)
    tl.utils = _mod("transformer_lens.utils", to_numpy=lambda t: t.detach().cpu().numpy())

    class _Float:
        def __class_getitem__(cls, item):
            return object

    _mod("jaxtyping", Float=_Float)
    _mod("wandb", init=lambda *a, **k: None, log=lambda *a, **k: None)
