"""crosscoder_amd — MI355X-native (gfx950 HIP) crosscoder training step.

Drop-in for mitroitskii/crosscoder-model-diff-replication's hot path: `CrossCoder`
(crosscoder.py), `Trainer.step` (trainer.py) and `Buffer.next` (buffer.py).  The directory
name is fixed by the build pipeline; import it as `crosscoder_amd` (see crosscoder_amd.py
at the repository root).
"""
from .crosscoder import CrossCoder, LossOutput, DTYPES  # noqa: F401
from .trainer import Trainer  # noqa: F401
from .buffer import Buffer, SyntheticBuffer  # noqa: F401
from .analysis import decoder_stats, fold_activation_scaling_factor, sae_vis_export  # noqa: F401

__version__ = "0.1.0"
