/* crosscoder_hip.h — C ABI of libcrosscoder_hip.so (gfx950 / MI355X).
 *
 * The drop-in boundary for ONE crosscoder training step (fwd + bwd + grad-clip + Adam) of
 * mitroitskii/crosscoder-model-diff-replication.  The reference has no FFI: its "operators"
 * are the torch calls inside CrossCoder / Trainer.  Each entry point below names the
 * reference code it replaces (file:line under the reference tree).
 *
 * Conventions
 *  - Every pointer is a DEVICE pointer (hipMalloc / torch tensor .data_ptr()), 16-byte aligned,
 *    row-major, rows contiguous.  The library never allocates or frees caller memory.
 *  - `dtype` selects the storage type of params / activations / grads: CC_BF16 or CC_F32
 *    (the reference's cfg["enc_dtype"] "bf16" / "fp32", crosscoder.py:12,30).
 *    All accumulations are fp32 (bf16 inputs go through bf16 MFMA with fp32 accumulate,
 *    fp32 inputs through the exact-f32 MFMA).
 *  - Shapes: B batch rows, n models, d d_model, h dict_size, K = n*d.
 *    Requirements: d % 8 == 0, h % 8 == 0 (16-byte vector rows); any B >= 1.  (The Python layer
 *    serves other dict_size / d_in on zero-padded dims: crosscoder_amd.engine.padded_dims.)
 *  - `stream` is a hipStream_t (torch.cuda.current_stream().cuda_stream); all launches are
 *    asynchronous on it.  No entry point synchronises, allocates, or keeps global state.
 *  - Return value: 0 = CC_OK, else a CC_ERR_* code (>= CC_ERR_HIP_BASE: hipError_t + base).
 *    cc_strerror() maps it to a message.
 *  - Partial-sum slabs ("*_part") are caller-allocated fp32 workspaces whose sizes come from
 *    cc_col_part_rows() / cc_wave_parts(); they make every reduction deterministic
 *    (fixed summation order, no float atomics).
 */
#ifndef CROSSCODER_HIP_H
#define CROSSCODER_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif
/* the library is built with -fvisibility=hidden: exactly the entry points declared here are exported */
#pragma GCC visibility push(default)

#define CC_BF16 1
#define CC_F32 2

#define CC_LAYOUT_KC 0 /* operand stored with the contraction index contiguous   */
#define CC_LAYOUT_MN 1 /* operand stored with the M (or N) index contiguous      */

enum {
  CC_OK = 0,
  CC_ERR_NULL = 1,
  CC_ERR_DTYPE = 2,
  CC_ERR_SHAPE = 3,
  CC_ERR_ALIGN = 4,
  CC_ERR_TOO_LARGE = 5,
  CC_ERR_HIP_BASE = 1000
};

int cc_version(void);
const char* cc_strerror(int code);

/* Workspace sizing.  Column-partial slabs written by GEMM epilogues have
 * cc_col_part_rows(M) rows of N floats; per-wave scalar partials have cc_wave_parts(M, N)
 * floats.  Row-block slabs of the elementwise kernels: cc_prep_part_rows(B) x K and
 * cc_loss_part_rows(B) x K; loss row stats: 2 * n * cc_loss_col_blocks(d) x B. */
int64_t cc_col_part_rows(int64_t M);
int64_t cc_wave_parts(int64_t M, int64_t N);    /* encode (B, h) per-wave partial count       */
int64_t cc_wgrad_parts(int64_t h, int64_t K, int dtype); /* wgrad_dec / wgrad_enc per-wave partials */
int64_t cc_prep_part_rows(int64_t B);
int64_t cc_loss_part_rows(int64_t B);
int64_t cc_loss_col_blocks(int64_t d);
int64_t cc_loss_scalars_len(int64_t B); /* floats in the `scalars` buffer of cc_loss_finalize */

/* Generic MFMA GEMM, fp32 output: C[M,N] = sum_k A(m,k) B(k,n).
 * a_layout KC: A at A[m*lda+k]; MN: A at A[k*lda+m].  b_layout KC: B at B[n*ldb+k];
 * MN: B at B[k*ldb+n].  (Test/diagnostic entry; the fused entries below use the same kernel.) */
int cc_gemm_f32out(const void* A, int a_layout, int64_t lda, const void* Bm, int b_layout, int64_t ldb,
                   float* C, int64_t ldc, int64_t M, int64_t N, int64_t K, int dtype, void* stream);

/* Buffer.next normalisation + CrossCoder.get_losses cast (buffer.py:115-124, crosscoder.py:99):
 * x_out[b, m*d+j] = dtype( float(x_in[b,m,j]) * float(factor[m]) ), factor may be NULL (=1).
 * in_dtype / factor_dtype in {CC_BF16, CC_F32}.  colsum_part (optional): per 64-row block
 * column sums of x_out -> reduced by cc_reduce_rows into x.mean(0) (crosscoder.py:112). */
int cc_prep_input(const void* x_in, int in_dtype, const void* factor, int factor_dtype, void* x_out,
                  float* colsum_part, int64_t B, int64_t n, int64_t d, int dtype, void* stream);
/* cc_prep_input that also stores x_t [n*d][B] = x_out^T (bf16 out, B % 8 == 0; x_t NULL -> cc_prep_input). */
int cc_prep_input_t(const void* x_in, int in_dtype, const void* factor, int factor_dtype, void* x_out, void* x_t,
                    float* colsum_part, int64_t B, int64_t n, int64_t d, int dtype, void* stream);

/* out[j] = scale * sum_{i<R} part[i*ld + j] (fixed order).  Optional: out_f32, out_t (dtype),
 * sq_part [cc_reduce_parts(C)] (per column block: sum of dtype-rounded out^2, for clip_grad_norm_),
 * dot_part [cc_reduce_parts(C)] (per column block: sum of out[j] * dot_w[j]; with out = the column
 * sums of acts and dot_w = the total decoder norms this is B * l1_loss, crosscoder.py:126). */
int cc_reduce_rows(const float* part, int64_t R, int64_t C, int64_t ld, float scale, float* out_f32,
                   void* out_t, int dtype, float* sq_part, const float* dot_w, float* dot_part, void* stream);
int64_t cc_reduce_parts(int64_t C);

/* W_dec.norm(dim=-1) and its sum over models (crosscoder.py:123-125):
 * norms[h*n + m] = ||W_dec[h,m,:]||_2, total[h] = sum_m norms, inv_norms (optional) = 1/norms
 * (0 where a norm is 0: the norm backward's masked value).  fp32 results. */
int cc_dec_norms(const void* W_dec, float* norms, float* total, float* inv_norms, int64_t h, int64_t n,
                 int64_t d, int dtype, void* stream);

/* CrossCoder.encode (crosscoder.py:69-80): acts[B,h] = act(x[B,K] . W_enc + b_enc), W_enc stored
 * h-major [h][K] (its physical layout, crosscoder.py:55-58).  act = ReLU if apply_relu.
 * Optional fused side outputs (NULL to skip), all from the dtype-rounded acts:
 *   colsum_part [cc_col_part_rows(B) x h]  column sums  (-> sum_b acts, for dL1/dW_dec)
 *   l1_part     [cc_wave_parts(B,h)]        sum acts*tn  (l1_loss numerator, crosscoder.py:126)
 *   l0_part     [cc_wave_parts(B,h)]        count acts>0 (l0_loss numerator, crosscoder.py:128) */
int cc_encode_fwd(const void* x, const void* W_enc, const void* b_enc, const float* tn, void* acts,
                  int apply_relu, float* colsum_part, float* l1_part, float* l0_part, int64_t B, int64_t K,
                  int64_t h, int dtype, void* stream);

/* A column reduction a GEMM launch can carry before its tiles -- cc_reduce_rows(part, rows, cols, ld, scale,
 * out_f32 = out) with the same bits -- so the step saves that launch: out[j] = scale * sum_{i<rows} part[i*ld + j]. */
typedef struct cc_colsum_job {
  const float* part;
  int64_t rows, cols, ld;
  float scale;
  float* out;
} cc_colsum_job;

/* 1 when cc_encode_fwd_t / cc_dacts_bwd_t / cc_wgrad_both_t serve a step of this shape and dtype. */
int cc_transposed_ok(int64_t B, int64_t K, int64_t h, int dtype);

/* cc_encode_fwd that also stores acts transposed, acts_t [h][B] (the batch-contiguous operand of
 * cc_wgrad_both_t).  bf16 with B, K, h % 8 == 0 (else CC_ERR_SHAPE).
 * mask_bits (optional, cc_mask_bits_words(B, h) u32): the activation mask (acts > 0) as 1 bit per element in
 * the GEMM's accumulator order, which cc_dacts_bwd_t reads instead of the acts tile (autograd of the ReLU,
 * crosscoder.py:77).
 * tile_ctr (optional): CC_TILE_CTR_WORDS u32, zero before the first launch that uses them and left zero by
 * every launch: the persistent launch then hands out its output tiles dynamically, per XCD, so workgroups
 * that start late (their CUs held by another stream's kernel) take fewer tiles; NULL: a static tile order.
 * The results are the same bits either way.  Launches sharing tile_ctr must be ordered (one stream).
 * pre (optional): a column reduction the launch runs first (the step: x.mean(0) from cc_prep_input_t's
 * column partials, crosscoder.py:112). */
#define CC_TILE_CTR_WORDS 8
int cc_encode_fwd_t(const void* x, const void* W_enc, const void* b_enc, const float* tn, void* acts, void* acts_t,
                    int apply_relu, float* colsum_part, float* l1_part, float* l0_part, uint32_t* mask_bits,
                    uint32_t* tile_ctr, const cc_colsum_job* pre, int64_t B, int64_t K, int64_t h, int dtype,
                    void* stream);

/* u32 words of cc_encode_fwd_t's mask_bits for a [B][h] activation (256 x 256 tiles x 512 threads x 4). */
int64_t cc_mask_bits_words(int64_t B, int64_t h);

/* CrossCoder.decode (crosscoder.py:82-89): recon = acts[B,h] . W_dec[h][K] (+ b_dec).
 * recon_f32 (optional): fp32 [B][K]; b_dec NULL -> partial sum without bias (latent-sharded use).
 * recon_t (optional): dtype [B][K] = dtype(acc + b_dec). */
int cc_decode_fwd(const void* acts, const void* W_dec, const void* b_dec, float* recon_f32, void* recon_t,
                  int64_t B, int64_t h, int64_t K, int dtype, void* stream);

/* cc_decode_fwd's fp32 partial reconstruction (no bias), scheduled for whole 256-tile waves: the
 * column blocks that fill whole waves run in one launch, the leftover tiles as S-way split-K passes
 * over caller workspace `ws` (cc_decode_ws_floats(B, h, K, dtype) floats; 0 = no split for this
 * shape, ws may then be NULL) summed in fixed order -- deterministic.  Same results as
 * cc_decode_fwd up to fp32 summation order in the leftover columns. */
int64_t cc_decode_ws_floats(int64_t B, int64_t h, int64_t K, int dtype);
int cc_decode_fwd_ws(const void* acts, const void* W_dec, float* recon_f32, float* ws, int64_t ws_floats, int64_t B,
                     int64_t h, int64_t K, int dtype, void* stream);

/* cc_decode_fwd_ws with W_dec given transposed, W_dec_t [K][h] (a copy the optimizer keeps, see
 * cc_adam_step_t): both operands then contract over h contiguously.  Same results. */
int cc_decode_fwd_ws_t(const void* acts, const void* W_dec_t, float* recon_f32, float* ws, int64_t ws_floats,
                       int64_t B, int64_t h, int64_t K, int dtype, void* stream);
/* cc_decode_fwd_ws (W_dec [h][K] read as stored) for the latent-sharded step's partial reconstruction
 * (crosscoder.py:82-89 without b_dec, summed over the ranks), carrying two small jobs so the step saves their
 * launches: pre (optional) -- a cc_colsum_job the launch runs before its tiles (the step's sum_b acts,
 * crosscoder.py:126, from G1's column partials) -- and, norm_part given, the decoder norms' finaliser
 * (cc_dec_norms_finalize(norm_part, h, n, d, norms, tn, inv_norms), d % 64 == 0) as extra blocks of the
 * split-K leftover's reduction launch.  recon_f32 bit-identical to cc_decode_fwd_ws; the jobs' outputs to
 * their stand-alone launches.  wait_ctr (optional, bf16): the launch first waits IN ITS KERNEL until
 * *wait_ctr - wait_target >= 0 (mod 2^32) -- the side-stream decoder-half Adam's done count, cc_adam_dec_norms --
 * instead of the stream waiting for that Adam's event, as cc_decode_loss does; past ~1 s it runs no tile and sets
 * *wait_err (host-visible), which the same step's cc_wgrad_both_sums_t (abort) turns into -inf squared sums. */
int cc_decode_partial(const void* acts, const void* W_dec, float* recon_f32, float* ws, int64_t ws_floats,
                      const float* norm_part, float* norms, float* tn, float* inv_norms, const cc_colsum_job* pre,
                      const uint32_t* wait_ctr, uint32_t wait_target, uint32_t* wait_err, int64_t B, int64_t h,
                      int64_t n, int64_t d, int dtype, void* stream);

/* get_losses reconstruction terms + their backward (crosscoder.py:104-121, autograd):
 * r = recon_f32 + b_dec; g_recon = dtype(grad_scale * (r - x)) with grad_scale = 2/B.
 * row_part [2][n*cc_loss_col_blocks(d)][B]: [0] sum (r-x)^2, [1] sum (x - x_mean)^2 per
 * (model, column block, row).  col_part [cc_loss_part_rows(B)][K]: column sums of g_recon. */
int cc_loss_fwd_bwd(const float* recon_f32, const void* b_dec, const void* x, const float* x_mean,
                    void* g_recon, float* row_part, float* col_part, float grad_scale, int64_t B, int64_t n,
                    int64_t d, int dtype, void* stream);
/* cc_loss_fwd_bwd over the batch rows [row0, row0 + rows) only (row0 % 32 == 0, row0 + rows <= B).
 * The slabs keep the whole-batch layout, so disjoint row ranges may be separate calls: the
 * latent-sharded step processes each batch slice as soon as its all-reduce has landed. */
int cc_loss_fwd_bwd_rows(const float* recon_f32, const void* b_dec, const void* x, const float* x_mean,
                         void* g_recon, float* row_part, float* col_part, float grad_scale, int64_t row0,
                         int64_t rows, int64_t B, int64_t n, int64_t d, int dtype, void* stream);
/* cc_loss_fwd_bwd_rows that also stores g_recon_t [n*d][B] = g_recon^T for its rows (bf16, B and rows
 * % 8 == 0; g_recon_t NULL -> cc_loss_fwd_bwd_rows). */
int cc_loss_fwd_bwd_rows_t(const float* recon_f32, const void* b_dec, const void* x, const float* x_mean,
                           void* g_recon, void* g_recon_t, float* row_part, float* col_part, float grad_scale,
                           int64_t row0, int64_t rows, int64_t B, int64_t n, int64_t d, int dtype, void* stream);

/* G2 + the reconstruction loss in one pass (crosscoder.py:82-89 then :104-121 and their autograd),
 * the fused form of cc_decode_fwd_ws_t + cc_loss_fwd_bwd_rows_t over all rows: the whole-contraction
 * tiles run the loss as their GEMM epilogue (the fp32 reconstruction never reaches HBM), the split-K
 * leftover columns are summed in cc_decode_fwd_ws's fixed order and then run the same arithmetic.
 * g_recon / g_recon_t are bit-identical to the two-call form; the partial slabs use other blocks:
 *   row_part [2][n * ncb][B], ncb = cc_decode_loss_ncb(..) = d / 64 column blocks per model
 *   col_part [cc_col_part_rows(B)][K] (column sums of g_recon per 128-row group)
 * so their sums agree to fp32 reassociation (cc_loss_tail / cc_loss_finalize_nb take ncb; the b_dec
 * gradient sums cc_col_part_rows(B) rows).  ws: cc_decode_ws_floats(B, h, n*d, dtype) floats.
 * bf16, B % 8 == 0, d % 64 == 0; cc_decode_loss_ncb returns 0 for shapes this entry does not serve. */
int64_t cc_decode_loss_ncb(int64_t B, int64_t h, int64_t n, int64_t d, int dtype);
int cc_decode_loss_t(const void* acts, const void* W_dec_t, const void* b_dec, const void* x, const float* x_mean,
                     float grad_scale, void* g_recon, void* g_recon_t, float* row_part, float* col_part, float* ws,
                     int64_t ws_floats, int64_t B, int64_t h, int64_t n, int64_t d, int dtype, void* stream);
/* cc_decode_loss_t reading W_dec [h][K] itself (the parameter, no transposed copy; same bits): the GEMM's B
 * operand goes through transposed LDS reads.  g_recon_t may be NULL here (not written then).
 * norm_part (optional, with norms / tn / inv_norms as in cc_dec_norms_finalize): the decoder norms'
 * finaliser rides in the launch of the split-K leftover (or runs right after the GEMM where the shape has
 * none) -- the same bits as cc_dec_norms_finalize(norm_part, h, n, d, norms, tn, inv_norms), ordered before
 * whatever the stream runs next (crosscoder.py:123-125 for the backward and the loss tail).
 * pre (optional): a column reduction the launch runs before its tiles (the step: sum_b acts from the
 * encoder's column partials, which G4 and the l1 loss read, crosscoder.py:126).
 * wait_ctr (optional): W_dec / b_dec / norm_part come from a producer on another stream (the decoder-half Adam,
 * cc_adam_dec_norms' done_ctr): every workgroup waits in the kernel, after `pre`, until
 * (int32_t)(*wait_ctr - wait_target) >= 0 instead of the stream waiting for an event.  A wait past ~1 s gives
 * up and sets *wait_err (host-visible memory, e.g. mapped pinned) -- the results are then invalid. */
int cc_decode_loss(const void* acts, const void* W_dec, const void* b_dec, const void* x, const float* x_mean,
                   float grad_scale, void* g_recon, void* g_recon_t, float* row_part, float* col_part, float* ws,
                   int64_t ws_floats, const float* norm_part, float* norms, float* tn, float* inv_norms,
                   const cc_colsum_job* pre, const uint32_t* wait_ctr, uint32_t wait_target, uint32_t* wait_err,
                   int64_t B, int64_t h, int64_t n, int64_t d, int dtype, void* stream);

/* Loss reduction (crosscoder.py:106-128, trainer.py:51-61): per-row explained variances
 * ev/ev_a/ev_b [B] (fp32) and scalars[0:8] = {l2, l1, l0, mean ev, mean ev_a, mean ev_b, 0, 0};
 * `scalars` holds cc_loss_scalars_len(B) floats (the tail is workspace).
 * l1_part [n_l1] / l0_part [n_l0]: partial sums of B * l1 (cc_reduce_rows dot_part, or the per-wave
 * partials of cc_encode_fwd) and of the active count (cc_encode_fwd), scaled by 1/B (NULL -> 0). */
int cc_loss_finalize(const float* row_part, const float* l1_part, int64_t n_l1, const float* l0_part, int64_t n_l0,
                     float* ev, float* ev_a, float* ev_b, float* scalars, float* l1l0_out, int64_t B, int64_t n,
                     int64_t d, void* stream);
/* (l1l0_out, optional: a second copy of scalars[1:3] -- the latent-sharded step all-reduces it) */
/* cc_loss_finalize that also writes scalars[0:8] to host_out[0:8] (mapped, coherent pinned host
 * memory, hipHostMallocMapped | hipHostMallocCoherent) and then, after a system-scope release,
 * the 32-bit word `seq` to host_out[8]: the host polls that word instead of a copy + event. */
int cc_loss_finalize_mapped(const float* row_part, const float* l1_part, int64_t n_l1, const float* l0_part,
                            int64_t n_l0, float* ev, float* ev_a, float* ev_b, float* scalars, float* l1l0_out,
                            float* host_out, uint32_t seq, int64_t B, int64_t n, int64_t d, void* stream);

/* cc_loss_finalize_mapped over a row_part of `ncb` column blocks per model (the producer's layout:
 * cc_loss_col_blocks(d) for cc_loss_fwd_bwd*, cc_decode_loss_ncb for cc_decode_loss_t).  host_out may
 * be NULL. */
int cc_loss_finalize_nb(const float* row_part, int64_t ncb, const float* l1_part, int64_t n_l1,
                        const float* l0_part, int64_t n_l0, float* ev, float* ev_a, float* ev_b, float* scalars,
                        float* l1l0_out, float* host_out, uint32_t seq, int64_t B, int64_t n, int64_t d, void* stream);

/* One launch for the forward's tail (crosscoder.py:106-128): the L1 dot partials
 * l1_part[j] = sum over the 64 latents of block j of colsum_acts * tn (colsum_acts [h] = sum_b acts,
 * formed by cc_reduce_rows from the encoder's column slab), the per-row EV terms of row_part (`ncb`
 * column blocks per model) and the loss scalars -- bit-identical to cc_reduce_rows(.., dot_w = tn,
 * dot_part = l1_part) followed by cc_loss_finalize_nb(.., n_l1 = cc_reduce_parts(h), ..).  Its
 * workgroups (256 threads, few registers, < 0.5 KB of LDS) fit beside a persistent GEMM launch's, so a
 * side stream can run it during the backward's first GEMM.  The last workgroup to finish runs the
 * scalar finaliser; `counter` is one device uint32, zero before the first call, left zero by every
 * call (launches sharing a counter must be ordered, e.g. one stream).  host_out may be NULL. */
int cc_loss_tail(const float* colsum_acts, const float* tn, int64_t h, float* l1_part, const float* row_part,
                 int64_t ncb, const float* l0_part, int64_t n_l0, float* ev, float* ev_a, float* ev_b, float* scalars,
                 float* l1l0_out, float* host_out, uint32_t seq, int64_t B, int64_t n, int64_t d, uint32_t* counter,
                 void* stream);

/* Backward through decode + L1 + ReLU (autograd of crosscoder.py:77,84-89,126):
 * g_pre[B,h] = (g_recon . W_dec^T + l1_scale * tn[h]) * (acts > 0),  l1_scale = l1_coeff / B.
 * colsum_part [cc_col_part_rows(B) x h]: column sums of g_pre (-> b_enc.grad). */
int cc_dacts_bwd(const void* g_recon, const void* W_dec, const void* acts, const float* tn, float l1_scale,
                 void* g_pre, float* colsum_part, int64_t B, int64_t K, int64_t h, int dtype, void* stream);

/* cc_dacts_bwd writing g_pre TRANSPOSED only: g_pre_t[j][b], row stride ldt >= B (a batch slice
 * [r0, r1) passes g_pre_t + r0 and B = r1 - r0).  bf16 with B, K, h, ldt % 8 == 0.
 * mask_bits (optional): cc_encode_fwd_t's mask bits of these rows (a slice starting at row r0, r0 % 256 == 0,
 * passes mask_bits + (r0 / 256) * cc_mask_bits_words(256, h)); used instead of reading the acts tile when
 * the shape takes the whole-tile form (B, h % 256 == 0), same bits.  tile_ctr: as cc_encode_fwd_t.
 * tail (optional): the forward's loss tail -- cc_loss_tail with these arguments, the same bits -- run by the
 * launch's first workgroups before their tiles (the last of them to finish runs the loss-scalar finaliser;
 * the tile counters then even out its late start). */
typedef struct cc_loss_tail_job {
  const float* colsum_acts;
  const float* tn;
  int64_t h;
  float* l1_part;
  const float* row_part;
  int64_t ncb;
  const float* l0_part;
  int64_t n_l0;
  float* ev;
  float* ev_a;
  float* ev_b;
  float* scalars;
  float* l1l0_out;
  float* host_out;
  uint32_t seq;
  int64_t B, n;
  uint32_t* counter;
} cc_loss_tail_job;
int cc_dacts_bwd_t(const void* g_recon, const void* W_dec, const void* acts, const float* tn, float l1_scale,
                   const uint32_t* mask_bits, void* g_pre_t, int64_t ldt, float* colsum_part, uint32_t* tile_ctr,
                   const cc_loss_tail_job* tail, int64_t B, int64_t K, int64_t h, int dtype, void* stream);

/* W_dec.grad [h][K] = acts^T . g_recon + l1_scale * sum_b(acts[:,h]) * W_dec[h,m,:]/||W_dec[h,m,:]||
 * (norm backward is 0 where the norm is 0; inv_norms from cc_dec_norms).
 * sq_part [cc_wgrad_parts(h,K,dtype)]: sum of grad^2. */
int cc_wgrad_dec(const void* acts, const void* g_recon, const void* W_dec, const float* inv_norms,
                 const float* colsum_acts, float l1_scale, void* grad_W_dec, float* sq_part, int64_t B,
                 int64_t h, int64_t n, int64_t d, int dtype, void* stream);

/* W_enc.grad, h-major [h][K] (the param's physical layout) = g_pre^T . x.  sq_part as above. */
int cc_wgrad_enc(const void* g_pre, const void* x, void* grad_W_enc, float* sq_part, int64_t B, int64_t h,
                 int64_t K, int dtype, void* stream);

/* cc_wgrad_dec and cc_wgrad_enc with the same arguments and results, as ONE launch when the
 * ping-pong GEMM serves them (bf16, K % 8 == 0): the two tile sets fill whole waves together
 * (2 x 1152 tiles = 9 x 256 CUs at config 2); otherwise two launches. */
int cc_wgrad_both(const void* acts, const void* g_recon, const void* W_dec, const float* inv_norms,
                  const float* colsum_acts, float l1_scale, void* grad_W_dec, float* sq_dec, const void* g_pre,
                  const void* x, void* grad_W_enc, float* sq_enc, int64_t B, int64_t h, int64_t n, int64_t d,
                  int dtype, void* stream);

/* cc_wgrad_both with the batch-major operands TRANSPOSED: actsT / g_preT [h][B], g_reconT / xT [K][B]
 * (the contraction index B contiguous), so both GEMMs read row-contiguous (KC) operand tiles.
 * Same outputs as cc_wgrad_both (same k order per output element). */
int cc_wgrad_both_t(const void* actsT, const void* g_reconT, const void* W_dec, const float* inv_norms,
                    const float* colsum_acts, float l1_scale, void* grad_W_dec, float* sq_dec, const void* g_preT,
                    const void* xT, void* grad_W_enc, float* sq_enc, int64_t B, int64_t h, int64_t n, int64_t d,
                    int dtype, void* stream);

/* clip_grad_norm_(params, max_norm) (trainer.py:46; torch/nn/utils/clip_grad.py): per-param
 * norms from the squared-sum partials sq[off[i] .. off[i+1]) (nparams <= 8, off on the HOST),
 * total = ||(norm_i)||, coef = min(1, max_norm / (total + 1e-6)).  emulate_bf16 rounds the
 * intermediate norms/coef to bf16 as torch does for bf16 grads.
 * out[0] = coef, out[1] = total norm, out[2 + i] = norm_i  (fp32, device). */
int cc_clip_finalize(const float* sq, const int64_t* off, int nparams, float max_norm, int emulate_bf16,
                     float* out, void* stream);

/* One launch for the backward's tail (trainer.py:45-46): the bias gradients
 * g_b_enc [h] = sum of gpre_colpart [R_enc x h], g_b_dec [K] = sum of loss_colpart [R_dec x K] (param
 * dtype) with their squared-sum partials sq_b_enc / sq_b_dec [cc_reduce_parts(.)] (which must be the
 * segments 2 and 3 of sq), then cc_clip_finalize over sq -- bit-identical to the two cc_reduce_rows
 * launches + cc_clip_finalize.  counter: as cc_loss_tail. */
int cc_grad_tail(const float* gpre_colpart, int64_t R_enc, int64_t h, void* g_b_enc, float* sq_b_enc,
                 const float* loss_colpart, int64_t R_dec, int64_t K, void* g_b_dec, float* sq_b_dec, int dtype,
                 const float* sq, const int64_t* off, int nparams, float max_norm, int emulate_bf16, float* clip_out,
                 uint32_t* counter, void* stream);
/* The end of the single-GPU backward (trainer.py:45-46) as ONE launch: cc_wgrad_both_t (dW_dec, dW_enc
 * + their sq partials) and cc_grad_tail (bias gradients + sq partials, clip_grad_norm_'s coefficient
 * into clip_out) -- the bias sums run before the GEMM tiles, the clip finaliser in the last workgroup
 * to finish.  Same outputs as cc_wgrad_both_t followed by cc_grad_tail (the clip coefficient up to
 * the order of its fp64 squared-sum accumulation).  nparams must be 4 (sq's segments W_enc, W_dec, b_enc,
 * b_dec); tile_sum: fp32 scratch of cc_wgrad_tile_sums(h, n*d) floats (each output tile's squared sum, which
 * the last workgroup adds in a fixed order: the coefficient's bits do not depend on which workgroup ran which
 * tile) followed by 4 uint64 words the launch accumulates -- shader-clock ticks, 100 MHz ticks and the launch
 * count over the lifetime of its last workgroup (the clock the chip held; zero them to start a window); tile_ctr:
 * as cc_encode_fwd_t.  abort_flag (optional, host-mapped or device word): when nonzero at the clip finaliser, clip_out[0] is
 * written as -1 (CC_CLIP_ABORTED: clip_grad_norm_'s coefficient is never negative) and every cc_adam_step /
 * cc_adam_dec_norms launch that reads that coefficient leaves p, m, v untouched -- the step's update is not applied
 * (the single-GPU step passes the word its G2 launch sets when its in-kernel wait times out).  Where the ping-pong
 * GEMM does not serve the shape (or dtype != bf16) it runs exactly those two entries. */
int64_t cc_wgrad_tile_sums(int64_t h, int64_t K);
int cc_wgrad_both_clip_t(const void* actsT, const void* g_reconT, const void* W_dec, const float* inv_norms,
                         const float* colsum_acts, float l1_scale, void* grad_W_dec, float* sq_dec, const void* g_preT,
                         const void* xT, void* grad_W_enc, float* sq_enc, int64_t B, int64_t h, int64_t n, int64_t d,
                         const float* gpre_colpart, int64_t R_enc, void* g_b_enc, float* sq_b_enc,
                         const float* loss_colpart, int64_t R_dec, void* g_b_dec, float* sq_b_dec, const float* sq,
                         const int64_t* off, int nparams, float max_norm, int emulate_bf16, float* clip_out,
                         uint32_t* counter, float* tile_sum, uint32_t* tile_ctr, const uint32_t* abort_flag, int dtype,
                         void* stream);
/* cc_wgrad_both_clip_t whose finaliser is cc_segment_sums instead of the clip (the latent-sharded step,
 * trainer.py:45-46 split across ranks): out[p] = the per-parameter squared sums, 0 where bit p of
 * zero_mask is set, to be all-reduced.  Equal to cc_wgrad_both_t + cc_grad_tail_sums (the sums up to the
 * order of their fp64 accumulation), which it runs itself where the ping-pong GEMM does not serve.  abort
 * (optional): the step's abort word (cc_decode_partial's wait_err); when set, out[p] = -inf for every p, so the
 * all-reduced sums carry the abort to every rank and cc_adam_step_clip (a negative sum) applies nothing. */
int cc_wgrad_both_sums_t(const void* actsT, const void* g_reconT, const void* W_dec, const float* inv_norms,
                         const float* colsum_acts, float l1_scale, void* grad_W_dec, float* sq_dec, const void* g_preT,
                         const void* xT, void* grad_W_enc, float* sq_enc, int64_t B, int64_t h, int64_t n, int64_t d,
                         const float* gpre_colpart, int64_t R_enc, void* g_b_enc, float* sq_b_enc,
                         const float* loss_colpart, int64_t R_dec, void* g_b_dec, float* sq_b_dec, const float* sq,
                         const int64_t* off, int nparams, int zero_mask, float* out, uint32_t* counter, float* tile_sum,
                         uint32_t* tile_ctr, const uint32_t* abort, int dtype, void* stream);
/* cc_grad_tail whose finaliser is cc_segment_sums instead of the clip (the latent-sharded step:
 * out[p] = the per-parameter squared sums, 0 where bit p of zero_mask is set, to be all-reduced). */
int cc_grad_tail_sums(const float* gpre_colpart, int64_t R_enc, int64_t h, void* g_b_enc, float* sq_b_enc,
                      const float* loss_colpart, int64_t R_dec, int64_t K, void* g_b_dec, float* sq_b_dec, int dtype,
                      const float* sq, const int64_t* off, int nparams, int zero_mask, float* out, uint32_t* counter,
                      void* stream);

/* Per-parameter sums of the squared-gradient partials, sq[off[p] .. off[p+1]) (nparams <= 8, off on
 * the HOST), for the latent-sharded step's all-reduce: out[p] = the sum (fp32), or 0 where bit p of
 * zero_mask is set (a replicated parameter counted on one rank only). */
int cc_segment_sums(const float* sq, const int64_t* off, int nparams, int zero_mask, float* out, void* stream);

/* torch.optim.Adam step (trainer.py:16-20,47; torch/optim/adam.py single-tensor path, no weight
 * decay / amsgrad) fused with the clip multiply: g' = dtype(g * coef[0]); m, v, p updated in place
 * over `numel` flat elements; step = the Adam step count AFTER increment; lr from LambdaLR.
 * dtype-rounding between torch's ops is reproduced (bf16 state like the reference).
 * max_blocks > 0: grid-stride over at most that many 256-thread workgroups (for an update that
 * runs beside a GEMM on another stream); 0: one pass, one 8-element chunk per thread.
 * coef[0] < 0 (CC_CLIP_ABORTED, see cc_wgrad_both_clip_t): nothing is updated (a done count still arrives). */
int cc_adam_step(void* p, const void* g, void* m, void* v, int64_t numel, const float* coef, double lr,
                 double beta1, double beta2, double eps, int64_t step, int64_t max_blocks, int dtype, void* stream);

/* cc_adam_step with clip_grad_norm_'s coefficient formed in the kernel from the per-parameter squared
 * gradient sums `sums` [nparams] (trainer.py:46 over parameters whose sums were combined elsewhere, e.g.
 * all-reduced over the latent shards): the arithmetic of cc_clip_finalize over one element per parameter.
 * clip_out (optional): [coef, total norm, per-parameter norms] as cc_clip_finalize writes them.  A negative
 * sum (an aborted step's -inf, cc_wgrad_both_sums_t's abort) makes the coefficient CC_CLIP_ABORTED: nothing is
 * updated. */
int cc_adam_step_clip(void* p, const void* g, void* m, void* v, int64_t numel, const float* sums, int nparams,
                      float max_norm, int emulate_bf16, float* clip_out, double lr, double beta1, double beta2,
                      double eps, int64_t step, int64_t max_blocks, int dtype, void* stream);

/* ---- around the step ---- */

/* Buffer.refresh's shuffle (buffer.py:111-113: buffer = buffer[randperm(rows)]): dst[i] = src[perm[i]]
 * for `rows` rows of `row_bytes` bytes (multiple of 16); perm: int64 device array (an index outside
 * [0, src_rows) gives a zero row).  dst must not overlap src. */
/* dst[c][r] = src[r][c] for 16-bit elements: src [rows][ld_src], dst [cols][ld_dst];
 * rows, cols, ld_src, ld_dst % 8 == 0.  (The step's batch-contiguous copies x^T and g_recon^T.) */
int cc_transpose_b16(const void* src, int64_t rows, int64_t cols, int64_t ld_src, void* dst, int64_t ld_dst,
                     void* stream);

/* W_dec_t [K][h] = W_dec^T plus the decoder norms of cc_dec_norms (same bits) from the same pass
 * over W_dec [h][K] (bf16; d % 64 == 0, h % 8 == 0).  part: cc_dec_norms_part_floats(h, n, d)
 * floats of workspace (per-row, per-64-column-block squared sums). */
int64_t cc_dec_norms_part_floats(int64_t h, int64_t n, int64_t d);
int cc_transpose_dec_norms(const void* W_dec, int64_t h, int64_t n, int64_t d, void* W_dec_t, float* part,
                           float* norms, float* total, float* inv_norms, void* stream);

/* The rest of cc_dec_norms from per-(row, 64-column block) squared sums (cc_adam_dec_transposed). */
int cc_dec_norms_finalize(const float* part, int64_t h, int64_t n, int64_t d, float* norms, float* total,
                          float* inv_norms, void* stream);

/* cc_adam_step over the decoder matrix W_dec [h][K] only (p/g/m/v point at W_dec in each arena; same
 * bits as cc_adam_step), in 64 x 64 tiles that also write W_dec_t = the updated W_dec^T and `part`
 * (cc_dec_norms_part_floats floats) for cc_dec_norms_finalize: the next step's decoder norms and G2
 * operand from the same HBM pass.  bf16, K % 64 == 0, h % 8 == 0; max_blocks caps the grid. */
/* The decoder half of Adam (trainer.py:47 over W_dec and b_dec: p/g/m/v point at the decoder half of each
 * arena, numel elements, W_dec [h][K] first; same bits as cc_adam_step / cc_adam_step_clip) that also writes
 * `part` (cc_dec_norms_part_floats(h, n, d) floats) from the updated W_dec for cc_dec_norms_finalize: the next
 * step's decoder norms (crosscoder.py:123-125, same bits as cc_dec_norms) without another pass over W_dec.
 * The clip coefficient comes from `coef`, or (sums != NULL) is formed from the per-parameter squared sums as
 * in cc_adam_step_clip.  K % 64 == 0; max_blocks caps the grid (0: 1024).
 * done_ctr (optional, max_blocks > 0): each of the launch's cc_adam_capped_blocks(numel, max_blocks)
 * workgroups adds 1 to *done_ctr once its stores are released (agent scope): the count a cc_decode_loss
 * launch on another stream waits for (wait_ctr / wait_target). */
int cc_adam_dec_norms(void* p, const void* g, void* m, void* v, int64_t numel, const float* coef, const float* sums,
                      int nparams, float max_norm, int emulate_bf16, double lr, double beta1, double beta2,
                      double eps, int64_t step, int64_t max_blocks, float* part, int64_t h, int64_t K, int dtype,
                      uint32_t* done_ctr, void* stream);
/* Workgroups of the capped-grid Adam launch (max_blocks > 0) over numel elements. */
int64_t cc_adam_capped_blocks(int64_t numel, int64_t max_blocks);

int cc_adam_dec_transposed(void* p, const void* g, void* m, void* v, int64_t h, int64_t K, const float* coef,
                           double lr, double beta1, double beta2, double eps, int64_t step, int64_t max_blocks,
                           void* W_dec_t, float* part, int dtype, void* stream);

int cc_gather_rows(const void* src, int64_t src_rows, const int64_t* perm, void* dst, int64_t rows,
                   int64_t row_bytes, void* stream);

/* fold_activation_scaling_factor (Crosscoder_model_diff.ipynb:35368-35378), in place:
 * W_enc[m] *= scale[m], W_dec[:, m] /= scale[m], b_dec[m] /= scale[m] (W_dec / b_dec may be NULL), each op
 * rounded to the parameter dtype like torch.  W_enc / W_dec in their [h][n*d] physical layout;
 * scale: n fp32 device values. */
int cc_fold_scaling(void* W_enc, void* W_dec, void* b_dec, const float* scale, int64_t h, int64_t n, int64_t d,
                    int dtype, void* stream);

/* Decoder-norm analytics (analysis.py:9-12,40), one pass over W_dec [h][n][d]:
 * norms[h*n + m] = ||W_dec[h,m]||; relative[h] = norms[h,1] / sum_m norms[h,m] (optional);
 * cosine[h] = <W_dec[h,0], W_dec[h,1]> / (norms[h,0] norms[h,1]) (optional).  fp32 outputs. */
int cc_decoder_stats(const void* W_dec, int64_t h, int64_t n, int64_t d, int dtype, float* norms, float* relative,
                     float* cosine, void* stream);

#pragma GCC visibility pop

#ifdef __cplusplus
}
#endif
#endif
