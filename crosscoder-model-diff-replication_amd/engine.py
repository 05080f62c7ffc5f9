"""The crosscoder training step as a fixed sequence of HIP launches over resident HBM buffers.

Data layout in HBM (one arena per role, all views of single allocations):
  params  [ W_enc h-major [h][K] | b_enc [h] | W_dec [h][K] | b_dec [K] ]   (dtype)
  grads   same layout (dtype)        exp_avg / exp_avg_sq   same layout (dtype)
  x [B][K], acts [B][h], g_recon [B][K] (dtype); recon [B][K] fp32 (latent-sharded step / two-pass form only).
  bf16 (transposed_wgrad): also x^T [K][B], acts^T [h][B], g_recon^T [K][B], and g_pre only as
  g_pre^T [h][B] -- G4/G5 contract over the batch, so these make both of their operands
  row-contiguous.  acts^T / g_pre^T come from G1's / G3's epilogues, x^T from the prep kernel, g_recon^T
  from G2's loss epilogue (LDS-staged transposed stores).  G2 reads W_dec [h][K] itself (transposed LDS
  reads of its B operand); the decoder norms come from the partial sums the decoder-half Adam writes.
W_enc's logical shape is [n, d, h] with strides (d, 1, K) exactly like the reference's
rearranged view (crosscoder.py:55-58), so both weight matrices are [h][K] row-major and
every GEMM streams 128-byte rows.

Step (reference trainer.py:41-63 -> crosscoder.py:96-130 -> autograd -> clip -> Adam), single GPU:
  prep      x = dtype(buf * factor), x^T, column sums for x.mean(0)          buffer.py:124, crosscoder.py:99
  G1        (prologue: x.mean(0)) acts = relu(x W_enc + b_enc), acts^T, mask bits, colsum/l0 slabs
                                                                            crosscoder.py:69-80,112,128
  (rest)    the decoder-half Adam's last rows of the previous step (+ their norm partials), then a wait
            for the side stream's rows
  G2+loss   (prologue: sum_b acts) acts W_dec + b_dec - x -> l2/tv row terms, g_recon = 2(r-x)/B,
            g_recon^T, db_dec slab (no fp32 reconstruction); its split-K leftover launch also finalises
            ||W_dec[h,m]||, their sum over m and inverses from the Adam's partials
                                                                            crosscoder.py:82-89,104-126
  G3        (prologue of its first workgroups: the loss tail -- l1 partials, EV, the loss scalars into
            mapped host memory) g_pre = (g_recon W_dec^T + l1c tn/B) * (acts>0), stored as g_pre^T
                                                                            crosscoder.py:106-128, autograd
  G4G5      dW_dec = acts^T g_recon + l1c/B colsum(acts) W_dec/||W_dec||,
            dW_enc = g_pre^T x, db_enc / db_dec, the clip coefficient        autograd, trainer.py:46
  adam      encoder half on this stream; the decoder half's first rows on the side stream beside the
            next step's G1 (with the next step's norm partials)              trainer.py:47
G1, G3 and G4G5 are persistent launches that hand out their tiles per XCD from counters (DYNAMIC_TILES).
"""
import contextlib

import torch

from . import _hip, ops

# Optional per-launch timer (bench.py installs one): an object with .span(name) -> context
# manager recording HIP events on torch's current stream around the launch.
TIMER = None


def _span(name):
    return TIMER.span(name) if TIMER is not None else contextlib.nullcontext()


# The persistent GEMMs (G1, G3, G4G5) hand out their tiles from per-XCD counters, so workgroups that start late
# (CUs held by the side stream's or RCCL's kernels) take fewer tiles; False: the static tile order.  The same
# bits either way (every partial-sum slot is indexed by tile; tests compare the two).
DYNAMIC_TILES = True


# The Trainer's loss tail rides in the backward's G3 launch (its first workgroups run it before their tiles, the
# dynamic tile order evens out their late start; cc_dacts_bwd_t's tail job), instead of a side-stream launch
# forked from the compute stream before G3.  The same bits either way.
LOSS_TAIL_IN_G3 = True


# G2 (the step's first reader of the decoder half) waits for the side-stream decoder-half Adam inside its kernel
# (a done counter the Adam's workgroups increment; cc_decode_loss' wait_ctr) instead of the compute stream
# waiting for the Adam's event: the ~10 us a cross-stream dependency takes to release the next kernel go away.
# Other readers still wait for the event.  The same bits either way.
G2_WAITS_IN_KERNEL = True


def _tile_ctr(ws, k):
    return ws.tile_ctr[k] if DYNAMIC_TILES else None


def padded_dims(h, d):
    """Kernel dims (h, d) of a crosscoder with dict_size h and d_in d: both rounded up to a multiple of 8
    (the kernels move 16-byte rows).  The padding latents / columns are zero in every arena and stay
    zero through the step (their pre-activations, reconstructions, gradients and Adam updates are 0),
    so the reference-shaped views see exactly the reference crosscoder."""
    return -(-h // 8) * 8, -(-d // 8) * 8


class Arena:
    """Flat storage for the four parameters (or their grads / Adam moments):
    [ W_enc h-major [h][K] | b_enc [h] | W_dec [h][K] | b_dec [K] ] -- the encoder half and the
    decoder half are contiguous, so Adam can update them as two launches (enc_part / dec_part).
    h, d are the kernel dims (padded_dims); ref = (dict_size, d_in) of the reference-shaped views
    when they differ."""

    def __init__(self, h, n, d, dtype, device, data=None, ref=None):
        self.h, self.n, self.d = h, n, d
        self.h_ref, self.d_ref = ref if ref is not None else (h, d)
        self.padded = (self.h_ref, self.d_ref) != (h, d)
        K = n * d
        self.K = K
        self.numel = 2 * h * K + h + K
        self.data = data if data is not None else torch.zeros(self.numel, dtype=dtype, device=device)
        o = 0
        self.W_enc_hk = self.data[o:o + h * K].view(h, K)
        o += h * K
        self.b_enc = self.data[o:o + h]
        o += h
        self.split = o  # enc_part = data[:split], dec_part = data[split:]
        self.W_dec_hk = self.data[o:o + h * K].view(h, K)
        o += h * K
        self.b_dec_flat = self.data[o:o + K]
        self.pending = None  # event the decoder half's Adam (side stream) records; see clip_and_adam
        # the decoder half's last rows, launched by the first reader on its own stream (engine.adam)
        self.pending_rest = None
        # a stream already ordered after `pending` by a launch that waited for the Adam in its kernel
        self.pending_ordered = None

    def enc_part(self):
        return self.data[:self.split]

    def dec_part(self):
        return self.data[self.split:]

    def wait_pending(self, kernel_wait=False):
        """Order torch's current stream after the decoder half's Adam if it ran on a side stream (launching
        its deferred last rows first, if any).  kernel_wait (the caller is a cc_decode_loss launch that can wait
        in its kernel): returns that wait's (counter, target) instead of ordering the stream, where the Adam
        signals one; the stream then counts as ordered once that launch is enqueued (pending_ordered)."""
        tok = None
        if self.pending_rest is not None:
            rest, self.pending_rest = self.pending_rest, None
            tok = rest(kernel_wait)
        if tok is not None:
            return tok
        if self.pending is not None:
            cur = torch.cuda.current_stream(self.data.device)
            if cur != self.pending_ordered:
                self.pending.wait(cur)
            self.pending = None
            self.pending_ordered = None
        return None

    def like(self, dtype=None, device=None):
        """A zeroed arena of the same dims (grads / Adam moments)."""
        return Arena(self.h, self.n, self.d, dtype or self.data.dtype, device or self.data.device,
                     ref=(self.h_ref, self.d_ref))

    # reference-shaped views ([:h_ref] latents, [:d_ref] columns per model of the kernel layout)
    def W_enc(self):  # [n, d, h], strides (d, 1, K)
        v = self.W_enc_hk.view(self.h, self.n, self.d)
        if self.padded:
            v = v[:self.h_ref, :, :self.d_ref]
        return v.permute(1, 2, 0)

    def W_dec(self):  # [h, n, d]
        v = self.W_dec_hk.view(self.h, self.n, self.d)
        return v[:self.h_ref, :, :self.d_ref] if self.padded else v

    def b_enc_ref(self):  # [h]
        return self.b_enc[:self.h_ref] if self.padded else self.b_enc

    def b_dec(self):  # [n, d]
        v = self.b_dec_flat.view(self.n, self.d)
        return v[:, :self.d_ref] if self.padded else v

    def views(self):
        return {"W_enc": self.W_enc(), "W_dec": self.W_dec(), "b_enc": self.b_enc_ref(), "b_dec": self.b_dec()}


class StepWorkspace:
    """All activations / partial-sum slabs of one step, allocated once per (B, shape, dtype)."""

    def __init__(self, B, n, d, h, dtype, device, transposed=None):
        f32 = torch.float32
        K = n * d
        self.B, self.n, self.d, self.h, self.K, self.dtype = B, n, d, h, K, dtype
        E = lambda *s, dt=f32: torch.empty(*s, dtype=dt, device=device)  # noqa: E731
        # batch-contiguous copies for the weight gradients (G4/G5 then read row-contiguous KC tiles on
        # both operands: ~20 % faster than the batch-major MN/MN form at config 2).  transposed=False
        # forces the batch-major form (same results; the parity test compares the two)
        self.tr = transposed_wgrad(B, K, h, dtype) if transposed is None else bool(transposed) and \
            transposed_wgrad(B, K, h, dtype)
        self.x = E(B, K, dt=dtype)
        self.x_t = E(K, B, dt=dtype) if self.tr else None
        self.x_colpart = E(ops.prep_part_rows(B), K)
        self.x_mean = E(K)
        self.norms = E(h, n)
        self.tn = E(h)
        self.acts = E(B, h, dt=dtype)
        # G2 + loss in one pass (decode_loss) when it serves the shape: its row terms come per 64-column
        # block and its b_dec-gradient partials per 128-row group; one storage holds either layout
        self.fused_ncb = ops.decode_loss_ncb(B, h, n, d, dtype) if self.tr else 0
        # the fused G2 reads W_dec [h][K] itself (transposed LDS reads); elsewhere in the transposed mode G2 reads
        # W_dec^T [K][h] (both operands h-contiguous), refreshed with the decoder norms after Adam
        self.W_dec_t = E(K, h, dt=dtype) if self.tr and not self.fused_ncb else None
        npart = ops.dec_norms_part_floats(h, n, d) if self.tr else 0
        # per-(row, 64-column block) squared sums of W_dec (d % 64 == 0): written by the decoder-half Adam
        # (cc_adam_dec_norms) or by the fused W_dec^T + norms pass
        self.norm_part = E(npart) if npart else None
        # the decoder-norm partials are complete but not yet finalised into norms / tn / inv_norms: the next G2
        # launch carries the finaliser (decode_loss), or flush_norms runs it before the first reader
        self.norms_fin_pending = False
        self.fork_events = [None, None]  # the step's last stream-fork events (loss tail, decoder-half Adam)
        self.tail_deferred = None  # (host, seq, l1l0_out) of a loss tail the G3 launch of the batch's last rows carries
        self.acts_t = E(h, B, dt=dtype) if self.tr else None
        # G1's activation mask as bits in the GEMM accumulator order: G3 reads 16 B per thread and tile instead
        # of the 128 KB acts tile (1/16 of the bytes, no LDS staging)
        self.mask_bits = E(ops.mask_bits_words(B, h), dt=torch.int32) if self.tr else None
        # G1's activation column-sum / l0 partial slabs, double-buffered: the loss tail that reads a
        # step's slabs runs on the side stream, which nothing orders before the NEXT step's G1 on torch's
        # stream; alternating slots orders every rewrite after that tail (the step after next waits for
        # this step's decoder-half Adam before G2, and the side stream runs the tail before that Adam)
        # (and the column sums reduced from them, which the side stream's loss tail reads: the NEXT step's
        # reduce runs on torch's stream before that step waits for the side stream)
        self._slots = [(E(ops.col_part_rows(B), h), E(ops.wave_parts(B, h)), E(h)) for _ in range(2)]
        self._slot = 1
        self.acts_colpart, self.l0_part, self.colsum_acts = self._slots[1]
        self.n_wave = ops.wave_parts(B, h)
        self.n_l1 = ops.reduce_parts(h)
        self.l1_part = E(self.n_l1)  # per 64-latent block: sum_h colsum_acts[h] * tn[h] (= B * l1)
        self.recon = E(B, K)
        nws = ops.decode_ws_floats(B, h, K, dtype)
        self.dec_ws = E(nws) if nws else None  # G2 split-K partials
        self.g_recon = E(B, K, dt=dtype)
        self.g_recon_t = E(K, B, dt=dtype) if self.tr else None
        self.ncb = ops.loss_col_blocks(d)
        rp = E(2 * n * max(self.ncb, self.fused_ncb) * B)
        self.row_part = rp[:2 * n * self.ncb * B].view(2, n * self.ncb, B)  # loss_fwd_bwd's layout
        self.row_part_fused = rp[:2 * n * self.fused_ncb * B].view(2, n * self.fused_ncb, B) if self.fused_ncb \
            else None
        # b_dec-gradient partial rows: the two-pass loss kernel writes one per 32 batch rows, the fused
        # G2 + loss epilogue one per 128-row wave half of every 256-row tile (more rows when B <= 32)
        self.loss_colpart = E(max(ops.loss_part_rows(B), ops.col_part_rows(B)), K)
        self.row_ncb = None         # layout of the row terms last written (None: loss_fwd_bwd's)
        self.loss_col_rows = ops.loss_part_rows(B)  # rows of loss_colpart last written
        self.ev = E(B)
        self.ev_a = E(B)
        self.ev_b = E(B)
        self.scalars = E(ops.loss_scalars_len(B))
        # transposed mode stores g_pre only as g_pre_t [h][B]; ws.g_pre is then its [B][h] view
        self.g_pre_t = E(h, B, dt=dtype) if self.tr else None
        self.g_pre = self.g_pre_t.t() if self.tr else E(B, h, dt=dtype)
        self.gpre_colpart = E(ops.col_part_rows(B), h)
        nw_w = ops.wgrad_parts(h, K, dtype)
        self.inv_norms = E(h, n)
        sizes = [nw_w, nw_w, ops.reduce_parts(h), ops.reduce_parts(K)]
        self.sq_off = [0]
        for s in sizes:
            self.sq_off.append(self.sq_off[-1] + s)
        self.sq = E(self.sq_off[-1])
        self.clip_out = E(8)
        self.tile_sum = E(ops.wgrad_tile_sums(h, K))  # per-tile squared sums of the fused G4G5 + grad tail
        ops.wgrad_clock(self.tile_sum).zero_()  # + the clock words the launch accumulates (bench: effective sclk)
        # per-XCD tile counters of the persistent G1 / G3 / G4G5 launches (dynamic tile order, DYNAMIC_TILES);
        # every launch leaves its counters at zero
        self.tile_ctr = torch.zeros(3, ops.TILE_CTR_WORDS, dtype=torch.int32, device=device)
        self.clip_ready = False  # backward(clip=...) already wrote clip_out (fused grad tail)
        self.acts_pending = False  # forward deferred the activation column sums to loss_finalize
        # arrival counters of the fused tail launches (loss tail, grad tail); each launch leaves 0
        self.tail_ctr = torch.zeros(2, dtype=torch.int32, device=device)
        # the side-stream decoder-half Adam's done counter (each workgroup adds 1; never reset) and the count
        # G2 waits for in its kernel (G2_WAITS_IN_KERNEL); wait_err: a mapped host word G2 sets if that wait
        # ever times out (checked by the next forward)
        self.adam_done = torch.zeros(8, dtype=torch.int32, device=device)
        self.adam_done_target = 0
        self.wait_err = None
        self.norms_token = None
        self.busy = None  # weakref to the token of an autograd graph whose backward still needs this workspace

    def next_slot(self):
        """Switch G1's partial slabs (acts_colpart, l0_part, colsum_acts) to the other slot (once per forward)."""
        self._slot ^= 1
        self.acts_colpart, self.l0_part, self.colsum_acts = self._slots[self._slot]

    def sq_slice(self, i):
        return self.sq[self.sq_off[i]:self.sq_off[i + 1]]


def transposed_wgrad(B, K, h, dtype):
    """Whether the step keeps batch-contiguous operand copies for G4/G5 (bf16 ping-pong shapes)."""
    return bool(ops.lib().cc_transposed_ok(B, K, h, ops.dtype_code(dtype)))


def _norms_token(P):
    # the decoder norms stay valid while W_dec is the same storage and has not been written in
    # place through torch (every such write bumps the view's version counter; our own Adam kernel
    # does not, and norms_for_next() is launched right after it)
    return (P.W_dec_hk.data_ptr(), P.W_dec_hk._version)


def norms_for_next(ws, P):
    """Launch the next step's decoder norms (and W_dec^T) now, right after Adam wrote W_dec, so they
    run while the host turns this step's loss scalars into the loss dict; forward() then skips them.
    (clip_and_adam(side_stream=...) launches them on the side stream itself.)"""
    if ws.norms_token == _norms_token(P):
        return
    _decoder_derived(ws, P)
    ws.norms_token = _norms_token(P)


def _decoder_derived(ws, P):
    if ws.W_dec_t is not None and ws.norm_part is not None:  # W_dec^T and the norms from one pass over W_dec
        with _span("dec_norms_T"):
            ops.transpose_dec_norms(P.W_dec_hk, ws.n, ws.d, ws.W_dec_t, ws.norm_part, ws.norms, ws.tn, ws.inv_norms)
        return
    if ws.W_dec_t is not None:
        ops.transpose(P.W_dec_hk, out=ws.W_dec_t)
    ops.dec_norms(P.W_dec_hk, ws.h, ws.n, ws.d, norms=ws.norms, total=ws.tn, inv_norms=ws.inv_norms)


def flush_norms(ws):
    """Finalise pending decoder norms on torch's current stream (where no G2 launch carried the finaliser)."""
    if ws.norms_fin_pending:
        ws.norms_fin_pending = False
        with _span("dec_norms"):
            ops.dec_norms_finalize(ws.norm_part, ws.h, ws.n, ws.d, ws.norms, ws.tn, ws.inv_norms)


def decoder_norms(ws, P):
    """||W_dec[h, m]||, their sum over m and inverses (crosscoder.py:123-125), unless still fresh."""
    if getattr(ws, "norms_token", None) == _norms_token(P):
        ws.norms_token = None  # consumed: W_dec changes with this step's Adam
        return
    ws.norms_token = None
    _decoder_derived(ws, P)


def forward(ws, P, x_in, factor=None, grad_scale=None, want_grad=True, loss=True, finalize=True):
    """Forward + reconstruction-loss gradient.  P: params Arena.  x_in [B, n, d] any of
    fp32/bf16, factor [n] or None.  Leaves losses in ws.scalars / ws.ev*, g_recon ready
    (loss=False: stops at the fp32 reconstruction, for loss_rows / loss_finalize by slices;
    finalize=False: stops after the loss rows, for loss_finalize_with_g3 / loss_finalize_beside).  Where the fused entry
    serves the shape, G2 and the loss rows are one pass (decode_loss_t; no fp32 reconstruction)."""
    B, n, d, h, K = ws.B, ws.n, ws.d, ws.h, ws.K
    ws.next_slot()
    with _span("prep"):
        ops.prep_input(x_in, factor, ws.dtype, out=ws.x, colsum_part=ws.x_colpart, out_t=ws.x_t)
    # G1 reads only the encoder half: it may overlap the previous step's decoder-half Adam.  x.mean(0) (first
    # read by the loss) and sum_b acts (G4's L1 term and the l1 loss, crosscoder.py:112,126): column reductions
    # of the prep / G1 partial slabs -- carried in the prologues of G1 and G2 where the step's fused path runs
    # (cc_colsum_job: no launches of their own), else two reduce_rows launches after G1
    fused = bool(loss and ws.fused_ncb)  # (fused_ncb: the transposed-operand step only)
    # (the latent-sharded step's G1 -- loss=False -- carries x.mean(0) too; its G2, decode_partial_jobs, carries
    # sum_b acts and the decoder norms' finaliser)
    x_job = ops.colsum_job(ws.x_colpart, ws.x_colpart.shape[0], K, 1.0 / B, ws.x_mean) if ws.tr else None
    with _span("G1_encode"):
        if ws.tr:
            ops.encode_fwd_t(ws.x, P.W_enc_hk, P.b_enc, ws.acts, ws.acts_t, True, colsum_part=ws.acts_colpart,
                             l0_part=ws.l0_part, mask_bits=ws.mask_bits, tile_ctr=_tile_ctr(ws, 0), pre=x_job)
        else:
            ops.encode_fwd(ws.x, P.W_enc_hk, P.b_enc, ws.acts, True, colsum_part=ws.acts_colpart,
                           l0_part=ws.l0_part)
    if x_job is None:
        ops.reduce_rows(ws.x_colpart, ws.x_colpart.shape[0], K, scale=1.0 / B, out_f32=ws.x_mean)
    acts_job = ops.colsum_job(ws.acts_colpart, ws.acts_colpart.shape[0], h, 1.0, ws.colsum_acts)
    fused_g2 = bool(loss and ws.fused_ncb)
    # the latent-sharded step's G2 (decode_partial_jobs: W_dec read as stored, bf16) waits in its kernel too
    partial_g2 = bool(not loss and ws.tr and ws.W_dec_t is None)
    # (only while the decoder norms are the Adam's own: otherwise decoder_norms below reads W_dec on this stream)
    wait = P.wait_pending(kernel_wait=(fused_g2 or partial_g2) and G2_WAITS_IN_KERNEL
                          and ws.norms_token == _norms_token(P))
    if wait is not None:
        wait = (*wait, _wait_err(ws))
    decoder_norms(ws, P)  # (+ W_dec^T), unless launched already after the last Adam
    if fused_g2:
        # (carries a pending norm finaliser and, fused, the activation column sums; waits in its kernel for the
        # side-stream Adam where `wait`)
        decode_loss(ws, P, grad_scale, pre=acts_job, wait=wait)
        ws.acts_pending = True
        if finalize:
            loss_finalize(ws)
        return
    with _span("G2_decode"):
        if ws.W_dec_t is not None:
            ops.reduce_rows(ws.acts_colpart, ws.acts_colpart.shape[0], h, out_f32=ws.colsum_acts)
            ops.decode_partial_t(ws.acts, ws.W_dec_t, ws.recon, ws.dec_ws)
        else:
            nf = (ws.norm_part, ws.norms, ws.tn, ws.inv_norms) if ws.norms_fin_pending else None
            ws.norms_fin_pending = False
            ops.decode_partial_jobs(ws.acts, P.W_dec_hk, ws.recon, ws.dec_ws, ws.n, ws.d, norm_fin=nf, pre=acts_job,
                                    wait=wait)
            if wait is not None:
                P.pending_ordered = torch.cuda.current_stream(ws.x.device)
    # (G2 does not read the norms: their finaliser after it, where the latent-sharded step's collective on the
    # reconstruction hides it)
    flush_norms(ws)
    # B * l1 = sum_h colsum_acts[h] * tn[h] (crosscoder.py:126) rides in the loss finaliser's launch
    # (loss_tail)
    ws.acts_pending = True
    if loss:
        loss_rows(ws, P, 0, ws.B, grad_scale)
        if finalize:
            loss_finalize(ws)


STEP_ABORTED_MSG = ("crosscoder_hip: the step was aborted -- G2's in-kernel wait for the previous step's decoder-half "
                    "Adam (side stream) timed out, so G2 ran none of its tiles and this step's Adam launches applied no "
                    "update (params and Adam moments are those before the step; its batch was consumed).  If that "
                    "Adam was still running when this step's backward wrote its gradients, the decoder half of the "
                    "previous update may be inconsistent: reload a checkpoint.")


def check_step_abort(ws):
    """Raise (once: the word is cleared) if a G2 launch of this workspace timed out in its in-kernel wait.  The
    step's clip finaliser (after G3, which wrote the loss scalars the host just read) still has to see the word, so
    the device is drained before it is cleared (an error path: the sync costs nothing that matters)."""
    if ws is not None and ws.wait_err is not None and ws.wait_err.u32[0]:
        torch.cuda.synchronize(ws.x.device)
        ws.wait_err.u32[0] = 0
        raise RuntimeError(STEP_ABORTED_MSG)


def _wait_err(ws):
    """The mapped host word a G2 launch sets if its in-kernel wait times out.  The Trainer raises in the same step
    (check_step_abort after its loss read); other callers see it here, at the next forward, at the latest."""
    if ws.wait_err is None:
        ws.wait_err = _hip.MappedHostBuffer(4)
    check_step_abort(ws)
    return ws.wait_err.device_ptr


def decode_loss(ws, P, grad_scale=None, pre=None, wait=None):
    """G2 + loss rows + g_recon (and g_recon^T) in one pass over the whole batch (decode_loss: W_dec read
    directly).  pre: an ops.colsum_job the launch runs first; wait: (counter, target, err) of the side-stream
    Adam it waits for in the kernel."""
    gs = 2.0 / ws.B if grad_scale is None else grad_scale
    nf = (ws.norm_part, ws.norms, ws.tn, ws.inv_norms) if ws.norms_fin_pending else None
    ws.norms_fin_pending = False
    with _span("G2_decode"):
        ops.decode_loss(ws.acts, P.W_dec_hk, P.b_dec_flat, ws.x, ws.x_mean, gs, ws.g_recon, ws.g_recon_t,
                        ws.row_part_fused, ws.loss_colpart, ws.dec_ws, ws.n, ws.d, norm_fin=nf, pre=pre, wait=wait)
    if wait is not None:
        P.pending_ordered = torch.cuda.current_stream(ws.x.device)
    ws.row_ncb = ws.fused_ncb
    ws.loss_col_rows = ops.col_part_rows(ws.B)


def loss_rows(ws, P, r0, r1, grad_scale=None):
    """Loss row terms + g_recon for batch rows [r0, r1) (r0 % 32 == 0); slabs keep the batch layout."""
    gs = 2.0 / ws.B if grad_scale is None else grad_scale
    with _span("loss"):
        ops.loss_fwd_bwd(ws.recon, P.b_dec_flat, ws.x, ws.x_mean, ws.g_recon, ws.row_part, ws.loss_colpart, gs, ws.B,
                         ws.n, ws.d, row0=r0, rows=r1 - r0, g_recon_t=ws.g_recon_t)
    ws.row_ncb = None
    ws.loss_col_rows = ops.loss_part_rows(ws.B)


def _row_part(ws):
    return ws.row_part if ws.row_ncb is None else ws.row_part_fused


def loss_colpart(ws):
    """The b_dec-gradient partial rows the last loss producer wrote."""
    return ws.loss_colpart[:ws.loss_col_rows]


def loss_finalize(ws, l1l0_out=None, host=None, seq=0):
    """Loss scalars / EV vectors.  After a forward (which left the l1 partials to be formed against the
    decoder norms) one launch does both (cc_loss_tail); a re-formed loss (same activations) only the
    finaliser.  host (a _hip.MappedHostBuffer): the scalars also land there, then `seq` in word 8."""
    flush_norms(ws)  # (no-op after forward(), which ran the finaliser with or before G2)
    ws.tail_deferred = None
    if ws.acts_pending:
        ops.loss_tail(ws.colsum_acts, ws.tn, ws.l1_part, _row_part(ws), ws.l0_part, ws.n_wave, ws.ev, ws.ev_a,
                      ws.ev_b, ws.scalars, ws.B, ws.n, ws.d, ws.tail_ctr[0:1], l1l0_out=l1l0_out, host=host, seq=seq,
                      ncb=ws.row_ncb)
        ws.acts_pending = False
        return
    ops.loss_finalize(_row_part(ws), ws.l1_part, ws.n_l1, ws.l0_part, ws.n_wave, ws.ev, ws.ev_a, ws.ev_b, ws.scalars,
                      ws.B, ws.n, ws.d, l1l0_out=l1l0_out, host=host, seq=seq,
                      ncb=ws.row_ncb if ws.row_ncb is not None else ops.loss_col_blocks(ws.d))


def loss_from_recon(ws, P, grad_scale=None):
    """Re-form g_recon (+ the loss slabs) for another grad_scale, from the forward's operands: after the
    fused pass (no fp32 reconstruction kept) G2 runs again on the same acts / W_dec^T."""
    if ws.row_ncb is not None:
        decode_loss(ws, P, grad_scale)
    else:
        loss_rows(ws, P, 0, ws.B, grad_scale)
    loss_finalize(ws)


def loss_finalize_beside(ws, side_stream, on_losses=None, host=None, seq=0):
    """loss_finalize (+ on_losses(ws.scalars), e.g. a host copy) on `side_stream`, after everything
    queued so far on torch's stream: the backward's G3 does not read the tail's outputs, so it starts
    right after the loss kernel (the tail's workgroups fit beside G3's), and nothing on torch's stream
    reads the tail's outputs (G4's activation column sums come from forward()).  host / seq: the scalars
    go straight to mapped host memory (loss_finalize); then no event is recorded and None is returned,
    else the event that marks the tail's end."""
    dev = ws.x.device
    # (device-scope events for every stream-to-stream hand-off of the step: a torch event's system-scope release
    # idles the recording stream ~1.7 us longer, profiles/r04_event_probe.txt)
    ready = _hip.DeviceEvent().record(torch.cuda.current_stream(dev))
    ws.fork_events[0] = ready  # (kept alive until the next step's fork: the side stream's wait references it)
    with torch.cuda.stream(side_stream):
        ready.wait(side_stream)
        loss_finalize(ws, host=host, seq=seq)
        if on_losses is not None:
            on_losses(ws.scalars)
        if host is not None and on_losses is None:
            return None
        return _hip.DeviceEvent().record(side_stream)


def loss_finalize_with_g3(ws, side_stream, host=None, seq=0):
    """The loss tail of loss_finalize(ws, host=host, seq=seq), carried by the backward's G3 launch where it serves the
    shape (LOSS_TAIL_IN_G3, the transposed-operand step); otherwise loss_finalize_beside on `side_stream`.  Returns
    None (G3 carries it; the host reads the scalars through `host`) or loss_finalize_beside's event."""
    if LOSS_TAIL_IN_G3 and ws.tr and ws.acts_pending and host is not None:
        ws.tail_deferred = (host, seq, None)
        return None
    return loss_finalize_beside(ws, side_stream, host=host, seq=seq)


def row_chunks(B, n_chunks):
    """Batch slices [r0, r1) for the chunked (comm-overlapped) step: boundaries on 256-row GEMM
    tiles, so each slice's d_acts launch owns whole column-partial rows."""
    step = -(-B // max(1, n_chunks))
    step = -(-step // 256) * 256
    return [(r0, min(B, r0 + step)) for r0 in range(0, B, step)]


def dacts_rows(ws, P, l1_coeff, r0, r1, l1_grad_weight=1.0):
    """G3 over batch rows [r0, r1) (r0 % 256 == 0): g_pre rows + their column-sum partial rows."""
    l1_scale = float(l1_coeff) * l1_grad_weight / ws.B
    c0, c1 = ops.col_part_rows(r0), ops.col_part_rows(r1)
    flush_norms(ws)
    tail = None
    # a deferred loss tail rides in the launch of the batch's LAST rows: every loss row is written by then (the
    # latent-sharded step's per-slice loss rows precede their slice's G3 on this stream)
    if ws.tail_deferred is not None and r1 == ws.B:
        host, seq, l1l0_out = ws.tail_deferred
        ws.tail_deferred = None
        if ws.tr:
            tail = ops.loss_tail_job(ws.colsum_acts, ws.tn, ws.l1_part, _row_part(ws), ws.l0_part, ws.n_wave, ws.ev,
                                     ws.ev_a, ws.ev_b, ws.scalars, ws.B, ws.n, ws.d, ws.tail_ctr[0:1],
                                     l1l0_out=l1l0_out, host=host, seq=seq, ncb=ws.row_ncb)
            ws.acts_pending = False
        else:
            loss_finalize(ws, l1l0_out=l1l0_out, host=host, seq=seq)
    with _span("G3_dacts"):
        if ws.tr:
            ops.dacts_bwd_t(ws.g_recon[r0:r1], P.W_dec_hk, ws.acts[r0:r1], ws.tn, l1_scale, ws.g_pre_t[:, r0:r1],
                            colsum_part=ws.gpre_colpart[c0:c1], mask_bits=ops.mask_bits_rows(ws.mask_bits, ws.h, r0, r1),
                            tile_ctr=_tile_ctr(ws, 1), tail=tail)
        else:
            ops.dacts_bwd(ws.g_recon[r0:r1], P.W_dec_hk, ws.acts[r0:r1], ws.tn, l1_scale, ws.g_pre[r0:r1],
                          colsum_part=ws.gpre_colpart[c0:c1])


def backward(ws, P, G, l1_coeff, l1_grad_weight=1.0, dacts_done=False, clip=None, sums_out=None, zero_mask=0,
             tail_done=None):
    """Gradients of l2 + l1_coeff * l1 into the grads Arena G (+ squared-sum partials).
    dacts_done: G3 already ran per batch slice (dacts_rows).  tail_done: the event of a loss tail
    running beside (loss_finalize_beside), waited for before G4.  clip (max_norm, single-GPU step): the
    bias-gradient sums and clip_grad_norm_'s coefficient in one launch (clip_and_adam then skips
    its clip_finalize).  sums_out (latent-sharded step): instead, the per-parameter squared sums in
    the same launch (segment_sums semantics, zero_mask), for the all-reduce."""
    B, n, d, h, K = ws.B, ws.n, ws.d, ws.h, ws.K
    l1_scale = float(l1_coeff) * l1_grad_weight / B
    # (a deferred decoder-half Adam launch of the last step reads the clip coefficient this launch rewrites)
    P.wait_pending()
    if not dacts_done:
        dacts_rows(ws, P, l1_coeff, 0, B, l1_grad_weight)
    if tail_done is not None:
        tail_done.wait(torch.cuda.current_stream(ws.x.device))
    if sums_out is not None and ws.tr:
        # G4 + G5 and the grad tail's per-parameter squared sums (for the all-reduce) in one launch
        with _span("G4G5_wgrad"):
            ops.wgrad_both_sums_t(ws.acts_t, ws.g_recon_t, P.W_dec_hk, ws.inv_norms, ws.colsum_acts, l1_scale,
                                  G.W_dec_hk, ws.sq_slice(1), ws.g_pre_t, ws.x_t, G.W_enc_hk, ws.sq_slice(0), n, d,
                                  ws.gpre_colpart, G.b_enc, ws.sq_slice(2), loss_colpart(ws), G.b_dec_flat,
                                  ws.sq_slice(3), ws.sq, ws.sq_off, sums_out, ws.tail_ctr[1:2], ws.tile_sum,
                                  zero_mask=zero_mask, tile_ctr=_tile_ctr(ws, 2),
                                  abort_ptr=ws.wait_err.device_ptr if ws.wait_err is not None else None)
        return
    if clip is not None and ws.tr:
        # G4 + G5 and the grad tail (bias sums + clip coefficient) in one launch
        with _span("G4G5_wgrad"):
            ops.wgrad_both_clip_t(ws.acts_t, ws.g_recon_t, P.W_dec_hk, ws.inv_norms, ws.colsum_acts, l1_scale,
                                  G.W_dec_hk, ws.sq_slice(1), ws.g_pre_t, ws.x_t, G.W_enc_hk, ws.sq_slice(0), n, d,
                                  ws.gpre_colpart, G.b_enc, ws.sq_slice(2), loss_colpart(ws), G.b_dec_flat,
                                  ws.sq_slice(3), ws.sq, ws.sq_off, clip, ws.dtype == torch.bfloat16, ws.clip_out,
                                  ws.tail_ctr[1:2], ws.tile_sum, tile_ctr=_tile_ctr(ws, 2),
                                  abort_ptr=ws.wait_err.device_ptr if ws.wait_err is not None else None)
        ws.clip_ready = True
        return
    with _span("G4G5_wgrad"):
        if ws.tr:
            ops.wgrad_both_t(ws.acts_t, ws.g_recon_t, P.W_dec_hk, ws.inv_norms, ws.colsum_acts, l1_scale,
                             G.W_dec_hk, ws.sq_slice(1), ws.g_pre_t, ws.x_t, G.W_enc_hk, ws.sq_slice(0), n, d)
        else:
            ops.wgrad_both(ws.acts, ws.g_recon, P.W_dec_hk, ws.inv_norms, ws.colsum_acts, l1_scale, G.W_dec_hk,
                           ws.sq_slice(1), ws.g_pre, ws.x, G.W_enc_hk, ws.sq_slice(0), n, d)
    if sums_out is not None:
        ops.grad_tail_sums(ws.gpre_colpart, G.b_enc, ws.sq_slice(2), loss_colpart(ws), G.b_dec_flat, ws.sq_slice(3),
                           ws.sq, ws.sq_off, sums_out, ws.tail_ctr[1:2], zero_mask=zero_mask)
        return
    if clip is not None:
        ops.grad_tail(ws.gpre_colpart, G.b_enc, ws.sq_slice(2), loss_colpart(ws), G.b_dec_flat, ws.sq_slice(3), ws.sq,
                      ws.sq_off, clip, ws.dtype == torch.bfloat16, ws.clip_out, ws.tail_ctr[1:2])
        ws.clip_ready = True
        return
    ops.reduce_rows(ws.gpre_colpart, ws.gpre_colpart.shape[0], h, out_t=G.b_enc, sq_part=ws.sq_slice(2))
    ops.reduce_rows(loss_colpart(ws), ws.loss_col_rows, K, out_t=G.b_dec_flat, sq_part=ws.sq_slice(3))


# workgroups of the decoder-half Adam that runs beside the next step's G1 (128 / 192 / 384 / 512 measured
# slower)
DEC_ADAM_BLOCKS = 256
# share of W_dec's rows whose Adam update runs on the side stream beside the next step's G1; the rest (and
# b_dec) runs on the main stream after G1 with the whole chip.  Beside G1 the
# side launch gets one wave per SIMD (G1 holds the rest of the register file), which streams slowly once
# G1 has finished.
DEC_SIDE_ROWS = 0.92
# False: the decoder half's Adam runs on torch's stream right after the encoder half, with the whole chip (no side
# stream, nothing deferred) -- the alternative DESIGN.md section 3.3 measures against the overlap with G1
DEC_ADAM_BESIDE_G1 = True
SERIAL_DEC_BLOCKS = 0  # (0: the library's default grid for the serial form)


def clip_and_adam(ws, P, G, M, V, lr, beta1, beta2, eps, step, max_norm=1.0, side_stream=None):
    """clip_grad_norm_ (from the squared-sum slabs of the backward) + Adam (see adam())."""
    emulate = ws.dtype == torch.bfloat16
    if not ws.clip_ready:
        ops.clip_finalize(ws.sq, ws.sq_off, max_norm, emulate, ws.clip_out)
    ws.clip_ready = False
    adam(ws, P, G, M, V, lr, beta1, beta2, eps, step, side_stream)


def adam(ws, P, G, M, V, lr, beta1, beta2, eps, step, side_stream=None, clip_sums=None):
    """Adam with the clip coefficient in ws.clip_out[0] -- or, clip_sums (sums [4], max_norm): formed in each
    launch from the per-parameter squared gradient sums (cc_adam_step_clip; the encoder-half launch also writes
    ws.clip_out), so no clip launch sits between the sums' all-reduce and Adam.  side_stream: the encoder half runs on torch's
    stream, then the decoder half (+ the next step's decoder norms / W_dec^T) on the side stream, so it
    overlaps the next step's prep / encoder GEMM (G1 reads only the encoder half); P.pending orders every
    later decoder-half use (forward() waits before G2; CrossCoder's accessors, FusedAdam.state and
    Trainer.synchronize() wait).  Without a side stream: one launch over the whole arena."""
    P.wait_pending()  # (no deferred rows of an earlier step may read this step's coefficient)
    coef = ws.clip_out[0:1]
    emulate = ws.dtype == torch.bfloat16

    def step_(p, g, m, v, max_blocks=0, clip_out=None):
        if clip_sums is None:
            ops.adam_step(p, g, m, v, coef, lr, beta1, beta2, eps, step, max_blocks=max_blocks)
        else:
            ops.adam_step_clip(p, g, m, v, clip_sums[0], clip_sums[1], emulate, lr, beta1, beta2, eps, step,
                               max_blocks=max_blocks, clip_out=clip_out)

    if side_stream is None:
        with _span("adam"):
            step_(P.data, G.data, M.data, V.data, clip_out=ws.clip_out)
        return
    dev = P.data.device
    with _span("adam"):
        step_(P.enc_part(), G.enc_part(), M.enc_part(), V.enc_part(), clip_out=ws.clip_out)
    if not DEC_ADAM_BESIDE_G1 and ws.W_dec_t is None and ws.norm_part is not None:
        # serial: the decoder half (+ the next step's norm partials) on this stream, the whole chip
        dec = [A.dec_part() for A in (P, G, M, V)]
        with _span("adam_dec"):
            ops.adam_dec_norms(*dec, ws.h, ws.K, lr, beta1, beta2, eps, step, ws.norm_part,
                               coef=coef if clip_sums is None else None, clip_sums=clip_sums, emulate=emulate,
                               max_blocks=SERIAL_DEC_BLOCKS)
        ws.norms_token = _norms_token(P)
        ws.norms_fin_pending = True
        return
    # both halves are HBM-bound: the decoder half starts after the encoder half (run together they only
    # share the bandwidth), i.e. beside the next step's prep / G1 on the main stream
    enc_done = _hip.DeviceEvent().record(torch.cuda.current_stream(dev))
    ws.fork_events[1] = enc_done
    with torch.cuda.stream(side_stream):
        enc_done.wait(side_stream)
        if ws.W_dec_t is None and ws.norm_part is not None:
            # the decoder norms' partials come out of the Adam launches themselves (no pass over W_dec of their
            # own).  The side stream updates the first hs rows of W_dec beside the next step's G1; the first
            # reader of the params (the next forward, after G1) launches the rest on its stream, waits for the
            # side part and forms the norms (P.pending_rest)
            K, nblk = ws.K, ws.K // 64
            hs = min(ws.h, int(ws.h * DEC_SIDE_ROWS) // 8 * 8)
            dec = [A.dec_part() for A in (P, G, M, V)]
            kw = dict(coef=coef if clip_sums is None else None, clip_sums=clip_sums, emulate=emulate)
            hp = (lr, beta1, beta2, eps, step)
            target = None
            if hs > 0:
                with _span("adam_dec"):
                    nb = ops.adam_dec_norms(*(t[:hs * K] for t in dec), hs, K, *hp, ws.norm_part[:hs * nblk],
                                            max_blocks=DEC_ADAM_BLOCKS, done_ctr=ws.adam_done, **kw)
                ws.adam_done_target = (ws.adam_done_target + nb) & 0xFFFFFFFF
                target = ws.adam_done_target
            done = _hip.DeviceEvent().record(side_stream)

            def rest(kernel_wait=False):
                # the rows on the reader's stream, then it waits for the side stream's rows; the norm partials are
                # then complete, and the finaliser rides in the next G2 launch (decode_loss: G3 and the loss tail,
                # its first readers, run after G2) or runs before the first other reader (flush_norms).
                # kernel_wait (the reader is that G2 launch): G2 waits for the side stream's rows in its kernel
                # (returns the done counter and its target; P.pending keeps the event for other streams' readers)
                cur = torch.cuda.current_stream(dev)
                with _span("adam_dec_rest"):
                    if ws.h > hs:
                        ops.adam_dec_norms(*(t[hs * K:] for t in dec), ws.h - hs, K, *hp, ws.norm_part[hs * nblk:],
                                           **kw)
                    else:  # (every row on the side stream: b_dec only)
                        step_(*(t[hs * K:] for t in dec))
                ws.norms_fin_pending = True
                if kernel_wait and target is not None:
                    P.pending = done
                    return ws.adam_done, target
                done.wait(cur)
                return None

            ws.norms_token = _norms_token(P)
            P.pending_rest = rest
            P.pending = None
            return
        else:
            with _span("adam_dec"):
                step_(P.dec_part(), G.dec_part(), M.dec_part(), V.dec_part(), max_blocks=DEC_ADAM_BLOCKS)
            norms_for_next(ws, P)
            done = _hip.DeviceEvent().record(side_stream)
    P.pending = done
