"""Latent (dictionary) sharding of the training step across ranks — one process per GPU,
RCCL (torch.distributed "nccl") over xGMI.

Rank r owns latents [r*h/G, (r+1)*h/G): its slice of W_enc / W_dec / b_enc and their Adam
moments; b_dec is replicated.  Per step (reference Trainer.step, trainer.py:41-63):
  1. every rank reads the SAME batch (replicated x), encodes its latents and decodes them into
     an fp32 partial reconstruction [B, n*d] (no bias)                     -> G1, G2 local
  2. all_reduce(SUM) of the partial reconstructions (the only bulk exchange: 4*B*n*d bytes),
     issued per batch slice (`recon_chunks`: 2 over several ranks, 1 on one) on RCCL's stream.
     As soon as slice c has landed, its loss rows / g_recon and its d_acts rows (G3) run on the
     compute stream while the all-reduce of slice c+1 is still on the wire, so only the first
     slice's all-reduce is exposed.  One slice is a synchronous collective on the compute stream.
     (Slicing the encode/decode instead would leave the 256-tile G2 launch a fraction of the 256
     CUs per slice: DESIGN.md section 6.)
  3. b_dec + loss + g_recon on the full reconstruction: identical on all ranks
  4. the rest of the backward is local (g_recon is replicated): G4, G5, db_enc local; db_dec
     replicated
  5. ONE small all-reduce: the per-parameter squared-gradient sums for clip_grad_norm_ (b_dec
     counted once) and the two latent-local loss sums (l1, l0)            24 bytes
  6. Adam on the local arena (b_dec updates are identical on every rank).

`ShardedStep` holds the orchestration (the collectives and how partial results combine) and
drives a backend that does the local compute: `HipShardBackend` (the product, engine.py
kernels on one GPU).  The CPU tests drive the same `ShardedStep` with a torch-CPU backend over
gloo to check the decomposition.
"""
import contextlib
import os
import warnings

import torch
import torch.distributed as dist

from . import engine, ops
from .buffer import fingerprint as buffer_fingerprint
from .crosscoder import CrossCoder, reference_init, write_checkpoint
from .trainer import reference_loss, rounded


def shard_range(h_total, world, rank):
    """Contiguous latent slice of `rank`; every shard keeps h % 8 == 0 (16-byte rows)."""
    if h_total % world:
        raise ValueError(f"dict_size {h_total} is not divisible by world size {world}")
    h = h_total // world
    if h % 8:
        raise ValueError(f"per-rank dict slice {h} must be a multiple of 8")
    return rank * h, (rank + 1) * h


def clip_sums_for_allreduce(sums, rank):
    """Per-parameter squared-gradient sums [W_enc, W_dec, b_enc, b_dec] of this rank, with the
    replicated b_dec term kept on rank 0 only so the all-reduced vector counts it once."""
    out = sums.clone()
    if rank != 0:
        out[3] = 0.0
    return out


def own_rows(B, world, rank, align=32):
    """Batch rows [r0, r1) whose loss this rank computes in the reduce-scatter exchange (`align`-row
    aligned: 32 = the HIP loss kernel's row blocks)."""
    if B % (align * world):
        raise ValueError(f"batch {B} must be a multiple of {align} x world ({align * world}) for "
                         "comm='reduce_scatter'")
    r = B // world
    return rank * r, (rank + 1) * r


class ShardedStep:
    """comm: how the partial reconstructions are combined.
      "all_reduce"      fp32 all-reduce of [B, n*d] in batch slices; each slice's loss and d_acts rows
                        run as it lands (2 x 4*B*n*d*(G-1)/G bytes per rank on the wire)
      "reduce_scatter"  fp32 reduce-scatter by batch rows -> loss on this rank's B/G rows -> bf16
                        all-gather of g_recon (+ the small loss partial slabs) -> d_acts on the whole
                        batch (4*B*n*d*(G-1)/G + 2*B*n*d*(G-1)/G bytes: 25 % fewer)."""

    def __init__(self, backend, group=None, comm="all_reduce"):
        if comm not in ("all_reduce", "reduce_scatter"):
            raise ValueError(f"comm must be 'all_reduce' or 'reduce_scatter', got {comm!r}")
        self.b = backend
        self.group = group
        self.comm = comm
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)

    def _combine_all_reduce(self, recon, l1c):
        b = self.b
        chunks = b.row_chunks()
        if len(chunks) == 1:
            # one slice: nothing to overlap, so a synchronous collective on the compute stream itself (torch
            # runs it there: no event hand-off to the collective stream and back, ~55 us on one GPU)
            with engine._span("exchange_wait0"):  # (bench attribution pass: the compute stream's time in it)
                dist.all_reduce(recon, op=dist.ReduceOp.SUM, group=self.group)
            b.rows_ready(0, recon.shape[0], l1c)
            return
        # every slice's all-reduce is queued at once on the collective stream; the compute stream
        # waits for slice c only when it needs it
        works = [dist.all_reduce(recon[r0:r1], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
                 for r0, r1 in chunks]
        for c, ((r0, r1), w) in enumerate(zip(chunks, works)):
            # (bench attribution pass: events around the wait on the compute stream = the time the compute stream
            # sits idle for slice c -- the exchange's exposed part)
            with engine._span(f"exchange_wait{c}"):
                w.wait()
            b.rows_ready(r0, r1, l1c)                # loss rows + g_recon + d_acts rows of the slice

    def _combine_reduce_scatter(self, recon, l1c):
        b = self.b
        r0, r1 = own_rows(recon.shape[0], self.world, self.rank, getattr(b, "row_align", 32))
        mine = b.own_recon_buffer(r1 - r0)
        with engine._span("exchange_wait0"):
            dist.reduce_scatter_tensor(mine, recon, op=dist.ReduceOp.SUM, group=self.group)
        b.loss_own_rows(mine, r0, r1)                # this rank's loss rows: g_recon rows, row terms
        pairs = b.gather_pairs(r0, r1, self.world)
        with engine._span("exchange_wait1"):
            for out, inp in pairs:
                dist.all_gather_into_tensor(out, inp, group=self.group)
        b.after_gather(l1c)                          # the whole batch's g_recon (+^T) -> d_acts (G3)

    def step(self, raw, factor, l1c, lr, betas, eps, t, max_norm=1.0, on_losses=None):
        """One step -> (scalars, red): the loss scalars (l1 / l0 of this rank's latents only) and the
        all-reduced [4 squared-gradient sums, l1, l0].  on_losses(scalars, red) is called once both
        are final on the device (before the clip / Adam launches; torch's current stream is then an
        auxiliary stream ordered after them)."""
        b = self.b
        recon = b.forward_partial(raw, factor)
        if self.comm == "all_reduce":
            self._combine_all_reduce(recon, l1c)
        else:
            self._combine_reduce_scatter(recon, l1c)
        red = b.reduce_buffer()                      # [6]: 4 clip sums + l1, l0 (latent-local)
        scalars = b.loss_finalize(red)               # [l2, l1, l0, ev, ev_a, ev_b, ...]; red[4:6] = local l1, l0
        b.backward(l1c, red, self.rank)              # red[0:4] = local squared sums (b_dec on rank 0 only)
        # one 24-byte collective for the squared sums and l1 / l0: a synchronous collective runs on torch's
        # current stream (no hand-off to the collective stream and back)
        with engine._span("sums_allreduce"):
            dist.all_reduce(red, op=dist.ReduceOp.SUM, group=self.group)
        if on_losses is not None:
            # the host copy from the backend's auxiliary stream (forked here, one event): the compute
            # stream goes straight on to the clip + Adam launches
            fork = getattr(b, "fork_aux", None)
            with (fork() if fork is not None else contextlib.nullcontext()):
                on_losses(scalars, red)
        b.clip_and_adam_from_sums(red[0:4], lr, betas, eps, t, max_norm)
        return scalars, red


class HipShardBackend:
    """Local compute of one rank on its GPU (engine.py kernels)."""

    def __init__(self, cc, recon_chunks=1, overlap_decoder_adam=True):
        self.cc = cc
        self.side = torch.cuda.Stream(device=cc.arena().data.device) if overlap_decoder_adam else None
        a = cc.arena()
        self.G = a.like()
        self.M = a.like()
        self.V = a.like()
        self.red = torch.zeros(6, dtype=torch.float32, device=a.data.device)
        self.recon_chunks = recon_chunks
        self.ws = None
        self._aux = None
        self._tail_carried = False  # this step's loss tail rode in the last d_acts launch (carry_tail)

    def fork_aux(self):
        """A stream other than the compute stream, ordered after the compute stream's work so far (one
        event); returns the context that makes it torch's current stream.  It is the side stream: idle
        between its decoder-half Adam + norms and this step's Adam (which it waits for next), and on a
        hardware queue of its own -- a stream created later may share the compute stream's queue (4 per
        process), where the host copies would sit in front of the Adam launch."""
        dev = self.cc.arena().data.device
        if self.side is not None:
            s = self.side
        else:
            if self._aux is None:
                self._aux = torch.cuda.Stream(device=dev)
            s = self._aux
        s.wait_stream(torch.cuda.current_stream(dev))
        return torch.cuda.stream(s)

    def forward_partial(self, raw, factor):
        cc = self.cc
        ws = self.ws = cc._workspace(raw.shape[0])
        # (a step that raised between carry_tail and loss_finalize must not leave the next step skipping its tail)
        self._tail_carried = False
        ws.tail_deferred = None
        engine.forward(ws, cc.arena(), cc.pad_input(raw), factor, loss=False)  # G1, norms, G2 -> fp32 partial recon
        return ws.recon

    def row_chunks(self):
        return engine.row_chunks(self.ws.B, self.recon_chunks)

    def carry_tail(self):
        """Let the d_acts launch of the batch's last rows carry the loss tail (l1 / l0 of this rank's latents into
        the step's reduce buffer, the scalars, the EVs): its first workgroups run it before their tiles, so the step
        has no loss-tail launch of its own (engine.LOSS_TAIL_IN_G3, as the single-GPU step)."""
        ws = self.ws
        if engine.LOSS_TAIL_IN_G3 and ws.tr and ws.acts_pending:
            ws.tail_deferred = (None, 0, self.red[4:6])
            self._tail_carried = True

    def rows_ready(self, r0, r1, l1c):
        P = self.cc.arena()
        engine.loss_rows(self.ws, P, r0, r1)
        if r1 == self.ws.B:
            self.carry_tail()
        engine.dacts_rows(self.ws, P, l1c, r0, r1)

    # ---- comm="reduce_scatter"
    def own_recon_buffer(self, rows):
        ws = self.ws
        if getattr(ws, "rs_recon", None) is None or ws.rs_recon.shape[0] != rows:
            ws.rs_recon = torch.empty(rows, ws.K, dtype=torch.float32, device=ws.x.device)
        return ws.rs_recon

    def loss_own_rows(self, mine, r0, r1):
        ws = self.ws
        ws.recon[r0:r1].copy_(mine)
        engine.loss_rows(ws, self.cc.arena(), r0, r1)  # g_recon rows, row terms, db_dec partial rows

    def gather_pairs(self, r0, r1, world):
        """(output, input) pairs for all_gather_into_tensor: g_recon rows (bf16), the db_dec partial rows
        (fp32, one per 32 batch rows) and the loss row terms (fp32 [2, n*ncb, B] slab, by columns)."""
        ws = self.ws
        p0, p1 = r0 // 32, r1 // 32
        rp = ws.row_part
        # gathered concatenated along dim 0 ([world * 2, n*ncb, rows]; gloo takes only that form)
        self._rp_all = torch.empty(world * rp.shape[0], rp.shape[1], r1 - r0, device=rp.device)
        return [(ws.g_recon, ws.g_recon[r0:r1].clone()),
                (ws.loss_colpart, ws.loss_colpart[p0:p1].clone()),
                (self._rp_all, rp[:, :, r0:r1].contiguous())]

    def after_gather(self, l1c):
        ws = self.ws
        rp = ws.row_part
        rp.copy_(self._rp_all.view(-1, rp.shape[0], rp.shape[1], self._rp_all.shape[2]).permute(1, 2, 0, 3)
                 .reshape(rp.shape))
        if ws.tr:
            ops.transpose(ws.g_recon, out=ws.g_recon_t)
        self.carry_tail()
        engine.dacts_rows(ws, self.cc.arena(), l1c, 0, ws.B)

    def loss_finalize(self, red):
        if self._tail_carried:  # (the last d_acts launch ran it, into red[4:6] = self.red[4:6])
            self._tail_carried = False
            if red is not self.red:
                raise RuntimeError("loss_finalize: the carried loss tail wrote l1 / l0 into the backend's own reduce "
                                   "buffer, not the one passed")
            return self.ws.scalars
        engine.loss_finalize(self.ws, l1l0_out=red[4:6])
        return self.ws.scalars

    def backward(self, l1c, red, rank):
        ws = self.ws
        # per-parameter squared sums straight into the all-reduce buffer (same launch as the bias
        # gradients); the replicated b_dec's counts on rank 0 only
        engine.backward(ws, self.cc.arena(), self.G, l1c, dacts_done=True, sums_out=red[0:4],
                        zero_mask=0 if rank == 0 else 1 << 3)

    def reduce_buffer(self):
        return self.red

    def clip_and_adam_from_sums(self, sums, lr, betas, eps, t, max_norm):
        # encoder half on this stream, decoder half + next step's norms on the side stream (engine.adam); each
        # launch forms clip_grad_norm_'s coefficient from the all-reduced sums itself (no clip launch between)
        engine.adam(self.ws, self.cc.arena(), self.G, self.M, self.V, lr, betas[0], betas[1], eps, t, self.side,
                    clip_sums=(sums, max_norm))


def shard_crosscoder(cfg, lo, hi, n_models=None):
    """This rank's CrossCoder: latents [lo, hi) of exactly the crosscoder `CrossCoder(cfg)` builds for
    the whole dictionary (reference crosscoder.py:31-62: the seeded CPU draws are made for all
    cfg["dict_size"] latents, then sliced), so a sharded run trains the reference's model."""
    n = int(n_models if n_models is not None else cfg.get("n_models", 2))
    W_dec = reference_init(cfg, n)[lo:hi]
    return CrossCoder(dict(cfg, dict_size=hi - lo), n_models=n, init_W_dec=W_dec)


class ShardedTrainer:
    """Trainer.step contract over latent shards (the whole job is one crosscoder with
    cfg["dict_size"] latents; this rank trains its slice)."""

    def __init__(self, cfg, buffer, group=None, crosscoder=None, recon_chunks=None, logger=None, comm="all_reduce"):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.cfg = cfg
        self.logger = logger
        lo, hi = shard_range(cfg["dict_size"], self.world, self.rank)
        self.lo, self.hi = lo, hi
        if crosscoder is None:
            crosscoder = shard_crosscoder(cfg, lo, hi)
        self.crosscoder = crosscoder
        self.buffer = buffer
        # batch slices of the exchange: one on a single rank (nothing to hide: a synchronous collective on
        # the compute stream), otherwise 2 -- the second slice's exchange hides under the first slice's
        # loss + d_acts, for a loss + d_acts launch pair and two stream hand-offs (~55 us,
        # profiles/r03_sharded_one_gpu.txt)
        chunks = recon_chunks if recon_chunks is not None else cfg.get("recon_chunks", 1 if self.world == 1 else 2)
        if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:
            # RCCL's streams take hardware queues of their own: with HIP's default 4 per process the side
            # stream can land on the compute stream's queue, and its decoder-half Adam then runs after the
            # encoder half instead of beside the next G1 (+~0.2 ms per step, profiles/r03_sharded_one_gpu.txt)
            warnings.warn("latent-sharded step: set GPU_MAX_HW_QUEUES=8 before the process touches the GPU "
                          "(streams may share hardware queues)", RuntimeWarning, stacklevel=2)
        self.backend = HipShardBackend(crosscoder, recon_chunks=chunks)
        self.engine = ShardedStep(self.backend, group, comm=comm)
        self.total_steps = cfg["num_tokens"] // cfg["batch_size"]
        self.step_counter = 0
        self.t = 0
        self.lr = cfg["lr"] * self.lr_lambda(0)
        self._host = None
        self.save_dir, self.save_version = None, 0  # rank 0's checkpoint directory (save())
        self._verified = None  # the buffer's refresh_count whose fingerprint the ranks last compared

    def lr_lambda(self, step):
        if step < 0.8 * self.total_steps:
            return 1.0
        return 1.0 - (step - 0.8 * self.total_steps) / (0.2 * self.total_steps)

    def get_l1_coeff(self):
        if self.step_counter < 0.05 * self.total_steps:
            return self.cfg["l1_coeff"] * self.step_counter / (0.05 * self.total_steps)
        return self.cfg["l1_coeff"]

    def _copy_losses(self, scalars, red):
        # pinned landing buffers, filled on the backend's auxiliary stream (ordered after the all-reduce of
        # the sums and l1 / l0): the host waits for the losses only, and the compute stream never waits for
        # the copy
        if self._host is None:
            self._host = torch.empty(8, dtype=torch.float32, pin_memory=True)
            self._host_red = torch.empty(6, dtype=torch.float32, pin_memory=True)
            self._copied = torch.cuda.Event()
        self._host.copy_(scalars[:8], non_blocking=True)
        self._host_red.copy_(red[:6], non_blocking=True)
        self._copied.record()

    def synchronize(self):
        """Order torch's current stream after the last step's side-stream (decoder-half) Adam."""
        self.crosscoder.arena().wait_pending()

    def _verify_buffer(self):
        # once per buffer state: at the first step and after every refresh (next_raw refreshes after slicing the
        # batch it returns, so each state is compared before the first batch taken from it)
        gen = getattr(self.buffer, "refresh_count", 0)
        if gen != self._verified:
            verify_replicated(self.buffer.fingerprint(), self.group, gen)
            self._verified = gen

    def step(self):
        whole = hasattr(self.buffer, "fingerprint")
        if whole:
            self._verify_buffer()
        raw, factor = self.buffer.next_raw()
        if whole:
            self._verify_buffer()
        else:  # (a batch source without the buffer protocol's fingerprint: every batch is compared, a host sync)
            verify_replicated(buffer_fingerprint(raw, factor), self.group, self.step_counter)
        l1c = self.get_l1_coeff()
        self.t += 1
        self.engine.step(raw, factor, l1c, self.lr, (self.cfg["beta1"], self.cfg["beta2"]), 1e-8, self.t,
                         on_losses=self._copy_losses)
        self.lr = self.cfg["lr"] * self.lr_lambda(self.t)
        self._copied.synchronize()
        if min(self._host_red[:4].tolist()) < 0:
            # a rank's G2 timed out in its in-kernel wait for its side-stream Adam: its squared sums came out -inf
            # (cc_wgrad_both_sums_t's abort), so the all-reduced sums made EVERY rank's Adam launches apply nothing
            # (cc_adam_step_clip); every rank rolls back its step count and LR and raises in this same step
            self.t -= 1
            self.lr = self.cfg["lr"] * self.lr_lambda(self.t)
            try:
                engine.check_step_abort(self.backend.ws)  # (clears this rank's word, if it was this rank's G2)
            except RuntimeError:
                pass
            raise RuntimeError(engine.STEP_ABORTED_MSG)
        s = self._host[:6].tolist()
        s[1], s[2] = self._host_red[4:6].tolist()  # l1, l0 over all ranks' latents
        # the reference's l1 / EV_A / EV_B are param-dtype tensors (crosscoder.py:115-126): same rounding as Trainer.step
        dt = self.crosscoder.dtype
        l1 = rounded(s[1], dt)
        d = {"loss": reference_loss(s[0], l1, l1c, dt), "l2_loss": s[0], "l1_loss": l1, "l0_loss": s[2],
             "l1_coeff": l1c, "lr": self.lr, "explained_variance": s[3], "explained_variance_A": rounded(s[4], dt),
             "explained_variance_B": rounded(s[5], dt)}
        self.step_counter += 1
        return d

    def log(self, loss_dict):
        if self.rank != 0:
            return
        if self.logger is not None:
            self.logger(loss_dict, self.step_counter)
        print(loss_dict)

    def save(self):
        """Gather every rank's slice on rank 0 and write ONE reference-format checkpoint there
        (crosscoder.py:132-146: checkpoints/version_N/{k}.pt + {k}_cfg.json, the full dictionary)."""
        sd = self.gather_state_dict(dst=0)
        if self.rank == 0:
            self.save_dir, self.save_version = write_checkpoint(sd, self.cfg, self.save_dir, self.save_version)
        dist.barrier(group=self.group)

    def train(self):
        """trainer.py:69-82 over the shards (logging and checkpoints on rank 0).  The reference saves in a
        `finally:` (trainer.py:81-82).  Here the save is a collective, so it must run where every rank leaves the
        loop at the SAME step.  SIGINT (torchrun forwards it to every rank, not necessarily between the same two
        collectives) therefore only sets a flag; every `stop_check_every` steps (cfg, default 10) the ranks agree
        on it with a one-word all_reduce(MAX) at a step boundary -- never inside a step's collectives, never
        between the two Adam halves -- then all of them save and raise KeyboardInterrupt.  Normal completion
        saves too.  Any other exception may be one rank's alone: a save would then wait forever for the others,
        so it propagates without the final checkpoint.  A second SIGINT on a rank whose flag is already set raises
        KeyboardInterrupt at once (no checkpoint): the way out of a rank stuck in a collective."""
        import signal
        import threading

        self.step_counter = 0
        stop = [False]
        prev = None
        def on_sigint(signum, frame):
            if stop[0]:
                signal.signal(signal.SIGINT, prev)
                raise KeyboardInterrupt
            stop[0] = True

        if threading.current_thread() is threading.main_thread():
            prev = signal.signal(signal.SIGINT, on_sigint)
        every = max(1, int(self.cfg.get("stop_check_every", 10)))
        interrupted = False
        try:
            for i in range(self.total_steps):
                loss_dict = self.step()
                if i % self.cfg["log_every"] == 0:
                    self.log(loss_dict)
                if (i + 1) % self.cfg["save_every"] == 0:
                    self.save()
                if (i + 1) % every == 0 and self.agree_stop(stop[0]):
                    interrupted = True
                    break
            # (a SIGINT after the last stop check: the ranks agree once more before the final save)
            if not interrupted and self.total_steps % every and self.agree_stop(stop[0]):
                interrupted = True
        finally:
            if prev is not None:
                signal.signal(signal.SIGINT, prev)
        self.save()
        if interrupted:
            raise KeyboardInterrupt

    def agree_stop(self, flag):
        """True on every rank if any rank's stop flag is set (a step-boundary collective of one word)."""
        return agree_stop(flag, self.group)

    def gather_state_dict(self, dst=None):
        return gather_state_dict(self.crosscoder, self.cfg["dict_size"], self.group, dst=dst)


REPLICA_MISMATCH_MSG = ("latent-sharded step: the ranks' activation buffers differ (fingerprint {lo} .. {hi} across "
                        "ranks after refresh {gen}) -- every rank must train on the same batch rows (SURVEY 8e): build "
                        "the Buffer with group=<the trainer's group> so that one harvest and one permutation are "
                        "shared, or give every rank an identically seeded SyntheticBuffer")


def verify_replicated(fp, group=None, gen=0):
    """Compare a fingerprint (buffer.fingerprint: the rows, their order and the normalisation factors) across the
    group's ranks -- one all_reduce(MIN) and one all_reduce(MAX) of two int64 words -- and raise on every rank if
    they differ (the all-reduced reconstruction would otherwise mix different batches silently)."""
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    lo, hi = fp.to(dev), fp.to(dev).clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    if not torch.equal(lo, hi):
        raise RuntimeError(REPLICA_MISMATCH_MSG.format(lo=lo.tolist(), hi=hi.tolist(), gen=gen))


def agree_stop(flag, group=None):
    """all_reduce(MAX) of one stop flag over the group: True on every rank if any rank's flag is set."""
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([1.0 if flag else 0.0], device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return t.item() > 0


def gather_state_dict(cc, h_total, group=None, dst=None):
    """Full reference-layout state_dict of a latent-sharded crosscoder (the ranks' latent slices
    concatenated; W_enc with the reference's strides (d, 1, n*d), b_dec from this rank -- it is replicated
    and identical on all ranks; padded kernel columns (d_in % 8 != 0) sliced off like Arena.views()).
    dst=None: all_gather, every rank gets the dict on its device.  dst=r: gathered one tensor at a time on
    rank r and moved to its host (no transient full-dictionary copy on the other ranks' GPUs); the other
    ranks return None."""
    a = cc.arena()
    a.wait_pending()
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n, d, d_ref = a.n, a.d, a.d_ref
    out = {}
    for name, t in (("W_dec", a.W_dec_hk), ("W_enc", a.W_enc_hk), ("b_enc", a.b_enc)):
        t = t.contiguous()
        if dst is None:
            parts = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(parts, t, group=group)
        else:
            parts = [torch.empty_like(t) for _ in range(world)] if rank == dst else None
            dist.gather(t, parts, dst=dist.get_global_rank(group, dst) if group is not None else dst, group=group)
            if rank != dst:
                continue
            parts = [p.cpu() for p in parts]
        out[name] = torch.cat(parts, 0)
        del parts
    if dst is not None and rank != dst:
        return None
    # compact reference strides (no copy when d_in % 8 == 0)
    W_dec = out["W_dec"].view(h_total, n, d)[:, :, :d_ref].contiguous()
    W_enc = out["W_enc"].view(h_total, n, d)[:, :, :d_ref].contiguous().permute(1, 2, 0)
    b_dec = a.b_dec().clone()
    if dst is not None:
        b_dec = b_dec.cpu()
    return {"W_enc": W_enc, "W_dec": W_dec, "b_enc": out["b_enc"], "b_dec": b_dec}
