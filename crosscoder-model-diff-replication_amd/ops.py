"""Tensor-level wrappers over the C ABI (include/crosscoder_hip.h).

Every function takes torch tensors that already live on a ROCm device, checks shapes on
the host, and launches on torch's current stream.  Nothing here computes on the CPU.
"""
import ctypes

import torch

from . import _lib
from ._lib import CC_BF16, CC_F32, CC_LAYOUT_KC, CC_LAYOUT_MN

_DT = {torch.bfloat16: CC_BF16, torch.float32: CC_F32}


def dtype_code(dtype):
    try:
        return _DT[dtype]
    except KeyError:
        raise TypeError(f"crosscoder_amd supports bf16 and fp32 storage, got {dtype}") from None


def lib():
    return _lib.load()


def _stream(t):
    if t.device.type != "cuda":
        raise RuntimeError(
            f"crosscoder_amd kernels run on a ROCm GPU; got a tensor on {t.device} "
            "(the CPU restatement lives in oracle/ and is test-only)")
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _vptr(p):
    """an optional raw device address (int, ctypes.c_void_p or None) as a c_void_p"""
    return p if isinstance(p, ctypes.c_void_p) else ctypes.c_void_p(p or 0)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


TILE_CTR_WORDS = 8  # CC_TILE_CTR_WORDS (include/crosscoder_hip.h)


def _ctr(t):
    """A persistent launch's per-XCD tile counters: int32 [TILE_CTR_WORDS] (zero; every launch leaves them zero),
    or None (static tile order)."""
    if t is None:
        return None
    if t.dtype != torch.int32 or t.numel() < TILE_CTR_WORDS:
        raise ValueError("tile counters: int32 tensor of at least TILE_CTR_WORDS elements")
    return _ptr(t)


def _contig(t, name):
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if t.data_ptr() % 16:
        raise ValueError(f"{name} must be 16-byte aligned")
    return t


def check(rc):
    _lib.check(rc)


# ---------------------------------------------------------------- sizing helpers
def col_part_rows(M):
    return int(lib().cc_col_part_rows(M))


def wave_parts(M, N):
    return int(lib().cc_wave_parts(M, N))


def wgrad_parts(h, K, dtype):
    return int(lib().cc_wgrad_parts(h, K, dtype_code(dtype)))


def prep_part_rows(B):
    return int(lib().cc_prep_part_rows(B))


def loss_part_rows(B):
    return int(lib().cc_loss_part_rows(B))


def loss_col_blocks(d):
    return int(lib().cc_loss_col_blocks(d))


def loss_scalars_len(B):
    return int(lib().cc_loss_scalars_len(B))


# ---------------------------------------------------------------- kernels
def gemm_f32out(A, a_layout, Bm, b_layout, M, N, K, out=None):
    """Generic MFMA GEMM (test/diagnostic): see cc_gemm_f32out."""
    lda = A.shape[-1]
    ldb = Bm.shape[-1]
    if out is None:
        out = torch.empty(M, N, device=A.device, dtype=torch.float32)
    check(lib().cc_gemm_f32out(_ptr(A), a_layout, lda, _ptr(Bm), b_layout, ldb, _ptr(out), out.shape[-1],
                               M, N, K, dtype_code(A.dtype), _stream(A)))
    return out


def prep_input(x_in, factor, dtype, out=None, colsum_part=None, out_t=None):
    """x_out[B, n*d] = dtype(x_in * factor[model]) (Buffer.next normalisation + get_losses cast);
    out_t (optional, bf16): also x_out^T [n*d, B]."""
    B, n, d = x_in.shape
    _contig(x_in, "x")
    if out is None:
        out = torch.empty(B, n * d, device=x_in.device, dtype=dtype)
    fdt = dtype_code(factor.dtype) if factor is not None else CC_F32
    if out_t is not None:
        if out_t.shape != (n * d, B) or not out_t.is_contiguous():
            raise ValueError("out_t must be a contiguous [n*d, B] tensor")
        check(lib().cc_prep_input_t(_ptr(x_in), dtype_code(x_in.dtype), _ptr(factor), fdt, _ptr(out), _ptr(out_t),
                                    _ptr(colsum_part), B, n, d, dtype_code(dtype), _stream(x_in)))
    else:
        check(lib().cc_prep_input(_ptr(x_in), dtype_code(x_in.dtype), _ptr(factor), fdt, _ptr(out),
                                  _ptr(colsum_part), B, n, d, dtype_code(dtype), _stream(x_in)))
    return out


def reduce_rows(part, R, C, scale=1.0, out_f32=None, out_t=None, sq_part=None, ld=None, dot_w=None, dot_part=None):
    dt = dtype_code(out_t.dtype) if out_t is not None else CC_F32
    check(lib().cc_reduce_rows(_ptr(part), R, C, C if ld is None else ld, scale, _ptr(out_f32), _ptr(out_t),
                               dt, _ptr(sq_part), _ptr(dot_w), _ptr(dot_part), _stream(part)))


def reduce_parts(C):
    return int(lib().cc_reduce_parts(C))


def dec_norms(W_dec_hk, h, n, d, norms=None, total=None, inv_norms=None):
    if norms is None:
        norms = torch.empty(h, n, device=W_dec_hk.device, dtype=torch.float32)
    if total is None:
        total = torch.empty(h, device=W_dec_hk.device, dtype=torch.float32)
    check(lib().cc_dec_norms(_ptr(W_dec_hk), _ptr(norms), _ptr(total), _ptr(inv_norms), h, n, d,
                             dtype_code(W_dec_hk.dtype), _stream(W_dec_hk)))
    return norms, total


def encode_fwd(x, W_enc_hk, b_enc, acts, apply_relu=True, tn=None, colsum_part=None, l1_part=None,
               l0_part=None):
    B, K = x.shape
    h = W_enc_hk.shape[0]
    check(lib().cc_encode_fwd(_ptr(x), _ptr(W_enc_hk), _ptr(b_enc), _ptr(tn), _ptr(acts), int(apply_relu),
                              _ptr(colsum_part), _ptr(l1_part), _ptr(l0_part), B, K, h, dtype_code(x.dtype),
                              _stream(x)))
    return acts


def mask_bits_words(B, h):
    return int(lib().cc_mask_bits_words(B, h))


def colsum_job(part, rows, cols, scale=1.0, out=None):
    """A column reduction a GEMM launch carries in its prologue (cc_colsum_job: reduce_rows(part, rows, cols,
    scale=scale, out_f32=out) with the same bits), passed by reference."""
    return ctypes.byref(_lib.ColsumJob(part.data_ptr(), rows, cols, part.stride(0) if part.dim() == 2 else cols,
                                       scale, out.data_ptr()))


def encode_fwd_t(x, W_enc_hk, b_enc, acts, acts_t, apply_relu=True, tn=None, colsum_part=None, l1_part=None,
                 l0_part=None, mask_bits=None, tile_ctr=None, pre=None):
    """encode_fwd that also stores acts_t [h][B] = acts^T (bf16, B % 8 == 0) and, optionally, the activation
    mask bits (int32 [mask_bits_words(B, h)]) that dacts_bwd_t reads instead of acts.  tile_ctr: int32
    [TILE_CTR_WORDS] zeroed counters -> dynamic per-XCD tile order (same bits).  pre: a colsum_job the launch
    runs first."""
    B, K = x.shape
    h = W_enc_hk.shape[0]
    if mask_bits is not None and mask_bits.numel() < mask_bits_words(B, h):
        raise ValueError("mask_bits too small")
    check(lib().cc_encode_fwd_t(_ptr(x), _ptr(W_enc_hk), _ptr(b_enc), _ptr(tn), _ptr(acts), _ptr(acts_t),
                                int(apply_relu), _ptr(colsum_part), _ptr(l1_part), _ptr(l0_part), _ptr(mask_bits),
                                _ctr(tile_ctr), pre, B, K, h, dtype_code(x.dtype), _stream(x)))
    return acts


def decode_fwd(acts, W_dec_hk, b_dec=None, recon_f32=None, recon_t=None):
    B, h = acts.shape
    K = W_dec_hk.shape[1]
    check(lib().cc_decode_fwd(_ptr(acts), _ptr(W_dec_hk), _ptr(b_dec), _ptr(recon_f32), _ptr(recon_t), B, h, K,
                              dtype_code(acts.dtype), _stream(acts)))


def decode_ws_floats(B, h, K, dtype):
    return int(lib().cc_decode_ws_floats(B, h, K, dtype_code(dtype)))


def decode_partial(acts, W_dec_hk, recon_f32, ws=None):
    """fp32 acts . W_dec without bias, whole-wave schedule + split-K leftover (cc_decode_fwd_ws)."""
    B, h = acts.shape
    K = W_dec_hk.shape[1]
    check(lib().cc_decode_fwd_ws(_ptr(acts), _ptr(W_dec_hk), _ptr(recon_f32), _ptr(ws),
                                 0 if ws is None else ws.numel(), B, h, K, dtype_code(acts.dtype), _stream(acts)))


def decode_partial_jobs(acts, W_dec_hk, recon_f32, ws, n, d, norm_fin=None, pre=None, wait=None):
    """decode_partial (the same recon_f32 bits) carrying the step's small jobs (cc_decode_partial): pre, an
    ops.colsum_job run before the tiles; norm_fin = (part, norms, total, inv_norms), the decoder norms' finaliser
    (dec_norms_finalize) as extra blocks of the split-K reduction launch; wait = (ctr, target, err_addr): the launch
    waits in the kernel for a done counter of adam_dec_norms on another stream (as decode_loss)."""
    B, h = acts.shape
    part, norms, total, inv = norm_fin if norm_fin is not None else (None, None, None, None)
    wctr, wtarget, werr = wait if wait is not None else (None, 0, None)
    check(lib().cc_decode_partial(_ptr(acts), _ptr(W_dec_hk), _ptr(recon_f32), _ptr(ws), 0 if ws is None else ws.numel(),
                                  _ptr(part), _ptr(norms), _ptr(total), _ptr(inv), pre, _ptr(wctr),
                                  int(wtarget) & 0xFFFFFFFF, werr, B, h, n, d, dtype_code(acts.dtype), _stream(acts)))


def decode_partial_t(acts, W_dec_t, recon_f32, ws=None):
    """decode_partial from the transposed decoder copy W_dec_t [K][h] (cc_decode_fwd_ws_t); same results."""
    B, h = acts.shape
    K = W_dec_t.shape[0]
    check(lib().cc_decode_fwd_ws_t(_ptr(acts), _ptr(W_dec_t), _ptr(recon_f32), _ptr(ws),
                                   0 if ws is None else ws.numel(), B, h, K, dtype_code(acts.dtype), _stream(acts)))


def decode_loss_ncb(B, h, n, d, dtype):
    """Row-term column blocks per model of decode_loss_t's row_part (d / 64), 0 if it does not serve the shape."""
    return int(lib().cc_decode_loss_ncb(B, h, n, d, dtype_code(dtype)))


def decode_loss_t(acts, W_dec_t, b_dec, x, x_mean, grad_scale, g_recon, g_recon_t, row_part, col_part, ws, n, d):
    """G2 + the reconstruction loss in one pass (cc_decode_loss_t): g_recon / g_recon_t bit-identical to
    decode_partial_t + loss_fwd_bwd(g_recon_t=...); row_part [2, n * d/64, B], col_part [B/128, K]."""
    B, h = acts.shape
    check(lib().cc_decode_loss_t(_ptr(acts), _ptr(W_dec_t), _ptr(b_dec), _ptr(x), _ptr(x_mean), grad_scale,
                                 _ptr(g_recon), _ptr(g_recon_t), _ptr(row_part), _ptr(col_part), _ptr(ws),
                                 0 if ws is None else ws.numel(), B, h, n, d, dtype_code(acts.dtype), _stream(acts)))


def decode_loss(acts, W_dec_hk, b_dec, x, x_mean, grad_scale, g_recon, g_recon_t, row_part, col_part, ws, n, d,
                norm_fin=None, pre=None, wait=None):
    """decode_loss_t reading W_dec [h, K] itself (cc_decode_loss, transposed LDS reads of the B operand): the same
    bits without the W_dec^T copy.  g_recon_t may be None.  norm_fin = (part, norms, total, inv_norms): the decoder
    norms' finaliser (dec_norms_finalize) rides in the launch.  wait = (ctr, target, err_addr): the launch waits in
    the kernel for a done counter of adam_dec_norms on another stream (err_addr: host-visible word set on a
    timeout)."""
    B, h = acts.shape
    part, norms, total, inv = norm_fin if norm_fin is not None else (None, None, None, None)
    wctr, wtarget, werr = wait if wait is not None else (None, 0, None)
    check(lib().cc_decode_loss(_ptr(acts), _ptr(W_dec_hk), _ptr(b_dec), _ptr(x), _ptr(x_mean), grad_scale,
                               _ptr(g_recon), _ptr(g_recon_t), _ptr(row_part), _ptr(col_part), _ptr(ws),
                               0 if ws is None else ws.numel(), _ptr(part), _ptr(norms), _ptr(total), _ptr(inv), pre,
                               _ptr(wctr), int(wtarget) & 0xFFFFFFFF, werr, B, h, n, d, dtype_code(acts.dtype),
                               _stream(acts)))


def loss_fwd_bwd(recon_f32, b_dec, x, x_mean, g_recon, row_part, col_part, grad_scale, B, n, d, row0=0, rows=None,
                 g_recon_t=None):
    """Loss terms + g_recon for batch rows [row0, row0 + rows) (default: all B rows);
    g_recon_t (optional, bf16 [n*d, B]): also those rows of g_recon^T."""
    rows = B - row0 if rows is None else rows
    if g_recon_t is not None:
        if g_recon_t.shape != (n * d, B) or not g_recon_t.is_contiguous():
            raise ValueError("g_recon_t must be a contiguous [n*d, B] tensor")
        check(lib().cc_loss_fwd_bwd_rows_t(_ptr(recon_f32), _ptr(b_dec), _ptr(x), _ptr(x_mean), _ptr(g_recon),
                                           _ptr(g_recon_t), _ptr(row_part), _ptr(col_part), grad_scale, row0, rows,
                                           B, n, d, dtype_code(x.dtype), _stream(x)))
        return
    check(lib().cc_loss_fwd_bwd_rows(_ptr(recon_f32), _ptr(b_dec), _ptr(x), _ptr(x_mean), _ptr(g_recon),
                                     _ptr(row_part), _ptr(col_part), grad_scale, row0, rows, B, n, d,
                                     dtype_code(x.dtype), _stream(x)))


def loss_finalize(row_part, l1_part, n_l1, l0_part, n_l0, ev, ev_a, ev_b, scalars, B, n, d, l1l0_out=None,
                  host=None, seq=0, ncb=None):
    """host (optional): a _hip.MappedHostBuffer that also receives scalars[0:8] and then `seq` in word 8.
    ncb: row_part's column blocks per model when it is not loss_fwd_bwd's layout (decode_loss_t's)."""
    if ncb is not None:
        check(lib().cc_loss_finalize_nb(_ptr(row_part), ncb, _ptr(l1_part), n_l1, _ptr(l0_part), n_l0, _ptr(ev),
                                        _ptr(ev_a), _ptr(ev_b), _ptr(scalars), _ptr(l1l0_out),
                                        host.device_ptr if host is not None else None, seq, B, n, d,
                                        _stream(row_part)))
        return
    if host is not None:
        check(lib().cc_loss_finalize_mapped(_ptr(row_part), _ptr(l1_part), n_l1, _ptr(l0_part), n_l0, _ptr(ev),
                                            _ptr(ev_a), _ptr(ev_b), _ptr(scalars), _ptr(l1l0_out), host.device_ptr,
                                            seq, B, n, d, _stream(row_part)))
        return
    check(lib().cc_loss_finalize(_ptr(row_part), _ptr(l1_part), n_l1, _ptr(l0_part), n_l0, _ptr(ev), _ptr(ev_a),
                                 _ptr(ev_b), _ptr(scalars), _ptr(l1l0_out), B, n, d, _stream(row_part)))


def loss_tail(colsum_acts, tn, l1_part, row_part, l0_part, n_l0, ev, ev_a, ev_b, scalars, B, n, d, counter,
              l1l0_out=None, host=None, seq=0, ncb=None):
    """The l1 dot partials from the reduced activation column sums + loss_finalize as one launch whose
    workgroups fit beside a persistent GEMM (cc_loss_tail; the same bits as reduce_rows(.., dot_part) +
    loss_finalize).  ncb: row_part's column blocks per model (default loss_fwd_bwd's layout)."""
    h = colsum_acts.numel()
    check(lib().cc_loss_tail(_ptr(colsum_acts), _ptr(tn), h, _ptr(l1_part), _ptr(row_part),
                             loss_col_blocks(d) if ncb is None else ncb, _ptr(l0_part), n_l0, _ptr(ev), _ptr(ev_a),
                             _ptr(ev_b), _ptr(scalars), _ptr(l1l0_out), host.device_ptr if host is not None else None,
                             seq, B, n, d, _ptr(counter), _stream(colsum_acts)))


def grad_tail(gpre_colpart, g_b_enc, sq_b_enc, loss_colpart, g_b_dec, sq_b_dec, sq, offsets, max_norm, emulate_bf16,
              out, counter):
    """The two bias-gradient reduce_rows (+ sq partials) + clip_finalize as one launch (same bits)."""
    arr = (ctypes.c_int64 * len(offsets))(*[int(o) for o in offsets])
    check(lib().cc_grad_tail(_ptr(gpre_colpart), gpre_colpart.shape[0], gpre_colpart.shape[1], _ptr(g_b_enc),
                             _ptr(sq_b_enc), _ptr(loss_colpart), loss_colpart.shape[0], loss_colpart.shape[1],
                             _ptr(g_b_dec), _ptr(sq_b_dec), dtype_code(g_b_enc.dtype), _ptr(sq), arr, len(offsets) - 1,
                             max_norm, int(emulate_bf16), _ptr(out), _ptr(counter), _stream(sq)))


def grad_tail_sums(gpre_colpart, g_b_enc, sq_b_enc, loss_colpart, g_b_dec, sq_b_dec, sq, offsets, out, counter,
                   zero_mask=0):
    """The two bias-gradient reduce_rows (+ sq partials) + segment_sums as one launch (same bits)."""
    arr = (ctypes.c_int64 * len(offsets))(*[int(o) for o in offsets])
    check(lib().cc_grad_tail_sums(_ptr(gpre_colpart), gpre_colpart.shape[0], gpre_colpart.shape[1], _ptr(g_b_enc),
                                  _ptr(sq_b_enc), _ptr(loss_colpart), loss_colpart.shape[0], loss_colpart.shape[1],
                                  _ptr(g_b_dec), _ptr(sq_b_dec), dtype_code(g_b_enc.dtype), _ptr(sq), arr,
                                  len(offsets) - 1, int(zero_mask), _ptr(out), _ptr(counter), _stream(sq)))


def segment_sums(sq, offsets, out, zero_mask=0):
    """out[p] = sum(sq[offsets[p]:offsets[p+1]]) (0 where bit p of zero_mask is set)."""
    arr = (ctypes.c_int64 * len(offsets))(*[int(o) for o in offsets])
    check(lib().cc_segment_sums(_ptr(sq), arr, len(offsets) - 1, int(zero_mask), _ptr(out), _stream(sq)))


def dacts_bwd(g_recon, W_dec_hk, acts, tn, l1_scale, g_pre, colsum_part=None):
    B, K = g_recon.shape
    h = W_dec_hk.shape[0]
    check(lib().cc_dacts_bwd(_ptr(g_recon), _ptr(W_dec_hk), _ptr(acts), _ptr(tn), l1_scale, _ptr(g_pre),
                             _ptr(colsum_part), B, K, h, dtype_code(g_recon.dtype), _stream(g_recon)))


def loss_tail_job(colsum_acts, tn, l1_part, row_part, l0_part, n_l0, ev, ev_a, ev_b, scalars, B, n, d, counter,
                  l1l0_out=None, host=None, seq=0, ncb=None):
    """loss_tail's arguments as a cc_loss_tail_job a d_acts launch carries (dacts_bwd_t(tail=...)), by reference."""
    p = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    return ctypes.byref(_lib.LossTailJob(
        p(colsum_acts), p(tn), colsum_acts.numel(), p(l1_part), p(row_part), loss_col_blocks(d) if ncb is None else ncb,
        p(l0_part), n_l0, p(ev), p(ev_a), p(ev_b), p(scalars), p(l1l0_out),
        host.device_ptr.value if host is not None else None, seq, B, n, p(counter)))


def dacts_bwd_t(g_recon, W_dec_hk, acts, tn, l1_scale, g_pre_t, colsum_part=None, mask_bits=None, tile_ctr=None,
                tail=None):
    """dacts_bwd storing g_pre transposed only: g_pre_t [h][>= B] view (column slice allowed, row stride
    g_pre_t.stride(0)).  mask_bits: encode_fwd_t's bits of these rows (see mask_bits_rows)."""
    B, K = g_recon.shape
    h = W_dec_hk.shape[0]
    if g_pre_t.shape[0] != h or g_pre_t.shape[1] != B or g_pre_t.stride(1) != 1:
        raise ValueError("g_pre_t must be an [h, B] view with unit column stride")
    if mask_bits is not None and mask_bits.numel() < mask_bits_words(B, h):
        raise ValueError("mask_bits too small")
    check(lib().cc_dacts_bwd_t(_ptr(g_recon), _ptr(W_dec_hk), _ptr(acts), _ptr(tn), l1_scale, _ptr(mask_bits),
                               _ptr(g_pre_t), g_pre_t.stride(0), _ptr(colsum_part), _ctr(tile_ctr), tail, B, K, h,
                               dtype_code(g_recon.dtype), _stream(g_recon)))


def mask_bits_rows(mask_bits, h, r0, r1):
    """The mask bits of batch rows [r0, r1) (r0 % 256 == 0) of encode_fwd_t's [B][h] bits."""
    if r0 % 256:
        raise ValueError("mask bits slices start on a 256-row tile")
    w = mask_bits_words(256, h)
    return mask_bits[(r0 // 256) * w:]


def transpose(src, out=None):
    """out [cols, rows] = src^T for a 2-D 16-bit tensor (rows, cols % 8 == 0); out may be a column slice view."""
    rows, cols = src.shape
    if src.element_size() != 2 or src.stride(1) != 1:
        raise ValueError("transpose: 2-D 16-bit tensor with unit column stride")
    if out is None:
        out = torch.empty(cols, rows, dtype=src.dtype, device=src.device)
    if out.shape != (cols, rows) or out.stride(1) != 1 or out.dtype != src.dtype:
        raise ValueError("transpose: out must be [cols, rows] of the same dtype, unit column stride")
    check(lib().cc_transpose_b16(_ptr(src), rows, cols, src.stride(0), _ptr(out), out.stride(0), _stream(src)))
    return out


def dec_norms_part_floats(h, n, d):
    return int(lib().cc_dec_norms_part_floats(h, n, d))


def transpose_dec_norms(W_dec_hk, n, d, W_dec_t, part, norms, total, inv_norms=None):
    """W_dec_t = W_dec^T and dec_norms' outputs (same bits) from one pass over W_dec (d % 64 == 0)."""
    h = W_dec_hk.shape[0]
    check(lib().cc_transpose_dec_norms(_ptr(W_dec_hk), h, n, d, _ptr(W_dec_t), _ptr(part), _ptr(norms), _ptr(total),
                                       _ptr(inv_norms), _stream(W_dec_hk)))


def dec_norms_finalize(part, h, n, d, norms, total, inv_norms=None):
    check(lib().cc_dec_norms_finalize(_ptr(part), h, n, d, _ptr(norms), _ptr(total), _ptr(inv_norms),
                                      _stream(part)))


def adam_dec_norms(p, g, m, v, h, K, lr, beta1, beta2, eps, step, part, coef=None, clip_sums=None, emulate=True,
                   max_blocks=0, done_ctr=None):
    """Adam over the decoder half p/g/m/v (flat views, W_dec [h, K] first) that also writes the decoder-norm
    partials of the updated W_dec into `part` (cc_adam_dec_norms; dec_norms_finalize completes them).
    coef: the clip coefficient tensor; or clip_sums = (sums, max_norm): formed in the kernel.  done_ctr (int32
    device word, max_blocks > 0): each workgroup adds 1 when its results are released; returns the number of
    workgroups (adam_capped_blocks) then, else None."""
    sums, max_norm = clip_sums if clip_sums is not None else (None, 0.0)
    check(lib().cc_adam_dec_norms(_ptr(p), _ptr(g), _ptr(m), _ptr(v), p.numel(), _ptr(coef), _ptr(sums),
                                  0 if sums is None else sums.numel(), float(max_norm), int(emulate), lr, beta1, beta2,
                                  eps, int(step), int(max_blocks), _ptr(part), h, K, dtype_code(p.dtype),
                                  _ptr(done_ctr), _stream(p)))
    return adam_capped_blocks(p.numel(), max_blocks) if done_ctr is not None else None


def adam_capped_blocks(numel, max_blocks):
    """Workgroups of the capped-grid Adam launch (cc_adam_capped_blocks)."""
    return int(lib().cc_adam_capped_blocks(int(numel), int(max_blocks)))


def adam_dec_transposed(p, g, m, v, coef, lr, beta1, beta2, eps, step, W_dec_t, part, max_blocks=0):
    """Adam over the decoder matrix p/g/m/v [h, K] (views into the arenas) + W_dec_t = p^T and the
    decoder-norm partials from the same pass."""
    h, K = p.shape
    check(lib().cc_adam_dec_transposed(_ptr(p), _ptr(g), _ptr(m), _ptr(v), h, K, _ptr(coef), lr, beta1, beta2, eps,
                                       int(step), int(max_blocks), _ptr(W_dec_t), _ptr(part), dtype_code(p.dtype),
                                       _stream(p)))


def wgrad_dec(acts, g_recon, W_dec_hk, norms, colsum_acts, l1_scale, grad, sq_part, n, d):
    B, h = acts.shape
    check(lib().cc_wgrad_dec(_ptr(acts), _ptr(g_recon), _ptr(W_dec_hk), _ptr(norms), _ptr(colsum_acts), l1_scale,
                             _ptr(grad), _ptr(sq_part), B, h, n, d, dtype_code(acts.dtype), _stream(acts)))


def wgrad_enc(g_pre, x, grad, sq_part):
    B, h = g_pre.shape
    K = x.shape[1]
    check(lib().cc_wgrad_enc(_ptr(g_pre), _ptr(x), _ptr(grad), _ptr(sq_part), B, h, K, dtype_code(g_pre.dtype),
                             _stream(g_pre)))


def wgrad_both(acts, g_recon, W_dec_hk, norms, colsum_acts, l1_scale, grad_dec, sq_dec, g_pre, x, grad_enc, sq_enc,
               n, d):
    """wgrad_dec + wgrad_enc (same results), one launch where the ping-pong GEMM serves both."""
    B, h = acts.shape
    check(lib().cc_wgrad_both(_ptr(acts), _ptr(g_recon), _ptr(W_dec_hk), _ptr(norms), _ptr(colsum_acts), l1_scale,
                              _ptr(grad_dec), _ptr(sq_dec), _ptr(g_pre), _ptr(x), _ptr(grad_enc), _ptr(sq_enc), B, h,
                              n, d, dtype_code(acts.dtype), _stream(acts)))


def wgrad_both_t(actsT, g_reconT, W_dec_hk, norms, colsum_acts, l1_scale, grad_dec, sq_dec, g_preT, xT, grad_enc,
                 sq_enc, n, d):
    """wgrad_both from transposed batch operands (actsT / g_preT [h][B], g_reconT / xT [n*d][B]); same results."""
    h, B = actsT.shape
    check(lib().cc_wgrad_both_t(_ptr(actsT), _ptr(g_reconT), _ptr(W_dec_hk), _ptr(norms), _ptr(colsum_acts), l1_scale,
                                _ptr(grad_dec), _ptr(sq_dec), _ptr(g_preT), _ptr(xT), _ptr(grad_enc), _ptr(sq_enc), B,
                                h, n, d, dtype_code(actsT.dtype), _stream(actsT)))


def wgrad_tile_sums(h, K):
    """floats of the per-tile squared-sum scratch of wgrad_both_clip_t / wgrad_both_sums_t (the tile sums, then the
    launch clock words: see wgrad_clock)"""
    return int(lib().cc_wgrad_tile_sums(h, K))


WGRAD_CLOCK_WORDS = 8  # floats at the end of the tile-sum scratch: 4 uint64 clock words (gemm.hip WgradTail::clock)


def wgrad_clock(tile_sum):
    """The clock words the fused G4G5 launches accumulate at the end of their tile-sum scratch, as a view
    [shader-clock ticks, 100 MHz ticks, launches, reserved] (int64; zero them to start a window).  The scratch is
    exactly cc_wgrad_tile_sums floats (_check_tile_sum), so the kernel's clock words are its last 8."""
    return tile_sum[-WGRAD_CLOCK_WORDS:].view(torch.int64)


def _check_tile_sum(tile_sum, h, K):
    # (exactly: the launch writes its clock words after the tile sums, and wgrad_clock reads the buffer's last 8)
    if tile_sum.dtype != torch.float32 or not tile_sum.is_contiguous() or tile_sum.numel() != wgrad_tile_sums(h, K):
        raise ValueError(f"tile_sum must be a contiguous fp32 buffer of exactly {wgrad_tile_sums(h, K)} floats "
                         f"(cc_wgrad_tile_sums({h}, {K})), got {tuple(tile_sum.shape)} {tile_sum.dtype}")


def wgrad_both_clip_t(actsT, g_reconT, W_dec_hk, norms, colsum_acts, l1_scale, grad_dec, sq_dec, g_preT, xT, grad_enc,
                      sq_enc, n, d, gpre_colpart, g_b_enc, sq_b_enc, loss_colpart, g_b_dec, sq_b_dec, sq, offsets,
                      max_norm, emulate_bf16, out, counter, tile_sum, tile_ctr=None, abort_ptr=None):
    """wgrad_both_t + grad_tail in one launch (the bias sums before the GEMM tiles, the clip coefficient
    in the last workgroup); same outputs.  abort_ptr: device address of the step's abort word (when set, out[0] is
    written as CLIP_ABORTED and the Adam launches reading it apply nothing)."""
    h, B = actsT.shape
    _check_tile_sum(tile_sum, h, n * d)
    arr = (ctypes.c_int64 * len(offsets))(*[int(o) for o in offsets])
    check(lib().cc_wgrad_both_clip_t(
        _ptr(actsT), _ptr(g_reconT), _ptr(W_dec_hk), _ptr(norms), _ptr(colsum_acts), l1_scale, _ptr(grad_dec),
        _ptr(sq_dec), _ptr(g_preT), _ptr(xT), _ptr(grad_enc), _ptr(sq_enc), B, h, n, d, _ptr(gpre_colpart),
        gpre_colpart.shape[0], _ptr(g_b_enc), _ptr(sq_b_enc), _ptr(loss_colpart), loss_colpart.shape[0], _ptr(g_b_dec),
        _ptr(sq_b_dec), _ptr(sq), arr, len(offsets) - 1, max_norm, int(emulate_bf16), _ptr(out), _ptr(counter),
        _ptr(tile_sum), _ctr(tile_ctr), _vptr(abort_ptr), dtype_code(actsT.dtype), _stream(actsT)))


CLIP_ABORTED = -1.0  # clip_out[0] of a step whose update was not applied (include/crosscoder_hip.h)


def wgrad_both_sums_t(actsT, g_reconT, W_dec_hk, norms, colsum_acts, l1_scale, grad_dec, sq_dec, g_preT, xT, grad_enc,
                      sq_enc, n, d, gpre_colpart, g_b_enc, sq_b_enc, loss_colpart, g_b_dec, sq_b_dec, sq, offsets, out,
                      counter, tile_sum, zero_mask=0, tile_ctr=None, abort_ptr=None):
    """wgrad_both_t + grad_tail_sums in one launch (the latent-sharded step); same outputs.  abort_ptr: device address
    of the step's abort word (when set, every out[p] is -inf: the all-reduced sums abort every rank's Adam)."""
    h, B = actsT.shape
    _check_tile_sum(tile_sum, h, n * d)
    arr = (ctypes.c_int64 * len(offsets))(*[int(o) for o in offsets])
    check(lib().cc_wgrad_both_sums_t(
        _ptr(actsT), _ptr(g_reconT), _ptr(W_dec_hk), _ptr(norms), _ptr(colsum_acts), l1_scale, _ptr(grad_dec),
        _ptr(sq_dec), _ptr(g_preT), _ptr(xT), _ptr(grad_enc), _ptr(sq_enc), B, h, n, d, _ptr(gpre_colpart),
        gpre_colpart.shape[0], _ptr(g_b_enc), _ptr(sq_b_enc), _ptr(loss_colpart), loss_colpart.shape[0], _ptr(g_b_dec),
        _ptr(sq_b_dec), _ptr(sq), arr, len(offsets) - 1, int(zero_mask), _ptr(out), _ptr(counter), _ptr(tile_sum),
        _ctr(tile_ctr), _vptr(abort_ptr), dtype_code(actsT.dtype), _stream(actsT)))


def clip_finalize(sq, offsets, max_norm, emulate_bf16, out):
    arr = (ctypes.c_int64 * len(offsets))(*[int(o) for o in offsets])
    check(lib().cc_clip_finalize(_ptr(sq), arr, len(offsets) - 1, max_norm, int(emulate_bf16), _ptr(out),
                                 _stream(sq)))


def adam_step(p, g, m, v, coef, lr, beta1, beta2, eps, step, max_blocks=0):
    check(lib().cc_adam_step(_ptr(p), _ptr(g), _ptr(m), _ptr(v), p.numel(), _ptr(coef), lr, beta1, beta2, eps,
                             int(step), int(max_blocks), dtype_code(p.dtype), _stream(p)))


def adam_step_clip(p, g, m, v, sums, max_norm, emulate_bf16, lr, beta1, beta2, eps, step, max_blocks=0,
                   clip_out=None):
    """adam_step with the clip coefficient formed in the kernel from per-parameter squared sums (fp32 [nparams])."""
    check(lib().cc_adam_step_clip(_ptr(p), _ptr(g), _ptr(m), _ptr(v), p.numel(), _ptr(sums), sums.numel(),
                                  float(max_norm), int(emulate_bf16), _ptr(clip_out), lr, beta1, beta2, eps, int(step),
                                  int(max_blocks), dtype_code(p.dtype), _stream(p)))


# ---------------------------------------------------------------- around the step
def gather_rows(src, perm, out=None):
    """out[i] = src[perm[i]] over dim 0 (Buffer.refresh's shuffle); perm int64 on the same device."""
    _contig(src, "src")
    if perm.dtype != torch.int64 or perm.device != src.device:
        raise ValueError("perm must be an int64 tensor on the source's device")
    rows = perm.numel()
    if out is None:
        out = torch.empty((rows,) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
    _contig(out, "out")
    row_bytes = src.element_size()
    for s_ in src.shape[1:]:
        row_bytes *= s_
    check(lib().cc_gather_rows(_ptr(src), src.shape[0], _ptr(perm.contiguous()), _ptr(out), rows, row_bytes,
                               _stream(src)))
    return out


def fold_scaling(W_enc_hk, W_dec_hk, b_dec_flat, scale, n, d):
    """In place W_enc[m] *= s[m], W_dec[:, m] /= s[m], b_dec[m] /= s[m] (scale: fp32 device [n];
    W_dec_hk / b_dec_flat may be None: encoder-only fold)."""
    h = W_enc_hk.shape[0]
    check(lib().cc_fold_scaling(_ptr(W_enc_hk), _ptr(W_dec_hk), _ptr(b_dec_flat), _ptr(scale), h, n, d,
                                dtype_code(W_enc_hk.dtype), _stream(W_enc_hk)))


def decoder_stats(W_dec_hk, n, d):
    """norms [h, n], relative norms [h], cosine similarities [h] (fp32) of W_dec."""
    h = W_dec_hk.shape[0]
    dev = W_dec_hk.device
    norms = torch.empty(h, n, device=dev, dtype=torch.float32)
    rel = torch.empty(h, device=dev, dtype=torch.float32)
    cos = torch.empty(h, device=dev, dtype=torch.float32)
    check(lib().cc_decoder_stats(_ptr(W_dec_hk), h, n, d, dtype_code(W_dec_hk.dtype), _ptr(norms), _ptr(rel),
                                 _ptr(cos), _stream(W_dec_hk)))
    return norms, rel, cos
