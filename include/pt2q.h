/*
 * pt2q.h — C ABI of the MI355X ternary PTQ calibration engine (libpt2q.so).
 *
 * The reference (shuhan-wang1/SNLP---Tenary-Post-train-Quantization) is pure PyTorch and has no
 * FFI; each entry point below replaces the reference operation cited next to it, and the
 * Python package (snlp---tenary-post-train-quantization_amd/) binds them with ctypes behind the
 * reference's own class surface.
 *
 * Conventions
 *   - All tensor arguments are DEVICE pointers (HIP, gfx950) owned by the caller; nothing is
 *     retained after return.  Scratch comes from a caller-supplied workspace.
 *   - `stream` is a hipStream_t passed as void*; every call is stream-ordered and asynchronous
 *     (no host synchronisation, no allocation), so a caller may capture it into a hipGraph.
 *     The Cholesky inverse of an order m > 6144 (pt2q_cholesky_inverse, pt2q_quantize_layer)
 *     forks part of its work onto an internal low-priority stream (one per device and caller
 *     stream, created once) and joins it back with events before the call's last kernel: to the
 *     caller it is still one ordered sequence on `stream`, and under graph capture the side
 *     stream joins the capture.  PT2Q_CHOL_LOOKAHEAD=0 keeps everything on `stream`.
 *   - Matrices are row-major with explicit leading dimensions (in elements).
 *   - Return value: PT2Q_OK or an error code; launch-time argument errors only.  Numerical
 *     status discovered on the device (Cholesky breakdown) is written to `info_dev`; a stalled
 *     cross-workgroup wait is written to the workspace status word (PT2Q_E_STALL).
 *   - Arithmetic follows the PT2Q contract: results are bit-identical to the CPU
 *     oracle (oracle/pt2q_oracle.c) for every input.
 */
#ifndef PT2Q_H
#define PT2Q_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes */
#define PT2Q_OK 0
#define PT2Q_E_ARG 1
#define PT2Q_E_NOT_SPD 2 /* reported through info_dev; caller falls back to pinv (main.py:140) */
#define PT2Q_E_UNSUPPORTED 3
#define PT2Q_E_HIP 4
#define PT2Q_E_WORKSPACE 5
#define PT2Q_E_STALL 6     /* reported through the workspace status word (below), not returned */

/* Status word.  pt2q_gram (with a workspace), pt2q_quantize_layer, pt2q_quantize_blocks and
 * pt2q_ssr_select reserve the FIRST PT2Q_STATUS_BYTES of their workspace for an int status word,
 * zeroed on the call's stream.  Kernels that wait on another workgroup's hand-off (stream-K
 * Gram partials, the in-launch S1/d and top-k hand-offs) give up after a bounded number of polls
 * (seconds) and then set a non-zero bit there instead of continuing silently: after the stream
 * completes, a non-zero word means the outputs are invalid (PT2Q_E_STALL). */
#define PT2Q_STATUS_BYTES 256

/* element types */
#define PT2Q_F32 0
#define PT2Q_F16 1
#define PT2Q_BF16 2
#define PT2Q_I8 3

/* quantize flags */
#define PT2Q_FLAG_SSR 0x1          /* SSR block selection (reorder.py:107) instead of sequential */
#define PT2Q_FLAG_S1_GIVEN 0x2     /* one block (b >= m), PT2Q_AGA_ACT: A holds S1 (m floats) then d,
                                      from pt2q_s1_from_gram[_batched], instead of the Gram */
#define PT2Q_AGA_NONE 0x0          /* ATQ without activations (quantizer.py:274 X is None) */
#define PT2Q_AGA_ACT 0x10          /* variant M: S = X_bᵀX_b from the raw Gram (main.py:177) */
#define PT2Q_AGA_HESS 0x20         /* variant G: S = H_bbᵀH_bb from the damped Hessian (gptq.py:147) */
#define PT2Q_AGA_MASK 0x30

/* ATQ stage modes (quantizer.py per-method surface) */
#define PT2Q_STAGE_INIT 0   /* ternary_init            quantizer.py:32  */
#define PT2Q_STAGE_GRID 1   /* build_optimal_grid      quantizer.py:71  */
#define PT2Q_STAGE_ROUND 2  /* flexible_round          quantizer.py:110 */
#define PT2Q_STAGE_ITF 3    /* iterative_ternary_fitting quantizer.py:136 */
#define PT2Q_STAGE_AGA 4    /* activation_aware_grid_alignment quantizer.py:177 (given S1, d) */
#define PT2Q_STAGE_FULL 5   /* quantize                quantizer.py:250 (init+ITF[+AGA]) */

/* stage-timer classes (pt2q_stage_timing) */
#define PT2Q_TIMER_SETUP 0    /* W -> feature-major fp32 copy, counters, remaining set */
#define PT2Q_TIMER_SSR 1      /* similarity + top-k / sequential selection (reorder.py:107-143) */
#define PT2Q_TIMER_ATQ 2      /* ATQ init/ITF/AGA + S1/d + EF coefficients (quantizer.py:250-277) */
#define PT2Q_TIMER_EF 3       /* error feedback W[:, rem] -= E C (main.py:214) */
#define PT2Q_TIMER_OUT 4      /* result transposes (main.py:217-230) */
#define PT2Q_TIMER_GRAM 5     /* pt2q_gram / pt2q_gram_batched / the layer's Gram (main.py:128) */
#define PT2Q_TIMER_INVERSE 6  /* damping + Cholesky inverse, single or batched (main.py:129-139) */
#define PT2Q_TIMER_COUNT 7

const char* pt2q_version(void);
const char* pt2q_strerror(int status);

/* Workspace bytes needed by pt2q_quantize_layer / pt2q_quantize_blocks / pt2q_cholesky_inverse
 * for an n x m layer with block size b. */
size_t pt2q_layer_workspace_bytes(int n, int m, int b, int flags);
size_t pt2q_cholesky_workspace_bytes(int m);
/* The (smaller) workspace pt2q_quantize_blocks alone needs: status word + block-loop buffers. */
size_t pt2q_blocks_workspace_bytes(int n, int m, int b, int flags);

/* Measurement only (bench.py's live stage rooflines; no reference counterpart).  While enabled,
 * each stage of the block-loop entries (pt2q_quantize_blocks / _group / _layer) and every Gram /
 * Hessian-inverse entry brackets its launches with a pair of HIP events on its stream, tagged by
 * PT2Q_TIMER_* class.  pt2q_stage_timing(1) clears the log and enables it, (0) disables it;
 * pt2q_stage_timing_read waits for the recorded events and sums each class's elapsed
 * milliseconds into ms[0..nstages) (records: number of bracketed intervals).  One host thread, not
 * under graph capture.  With several streams in flight the intervals overlap other streams' work,
 * so a caller wanting kernel-busy times runs one stream. */
int pt2q_stage_timing(int enable);
int pt2q_stage_timing_read(double* ms, int nstages, int* records);

/* G = XᵀX (accumulate=0), G = G + XᵀX (accumulate=1), or continue (accumulate=2): every
 * entry's chain resumes from G, so Grams streamed batch by batch are bit-identical to one Gram
 * of the concatenated rows.  X: N x m of type xdtype (X may be NULL when N = 0).
 * Arithmetic: f32 X -> k-ascending fmaf chains (f32 MFMA); fp16 / bf16 X -> the 16-bit MFMA
 * chain (v_mfma_f32_32x32x16_*: rows in groups of 8, one rounding per group; restated by
 * oracle orc_gram16), for which the continue guarantee needs every batch but the last to have
 * a multiple of 8 rows.
 * Replaces main.py:128 (H = X.T @ X over the captured activations, main.py:293),
 * gptq.py:59-76 (GPTQ.add_batch, accumulate=1). Writes the full symmetric matrix.
 * workspace (nullable, pt2q_gram_workspace_bytes(m)) enables the balanced split over all CUs. */
size_t pt2q_gram_workspace_bytes(int m);
int pt2q_gram(const void* X, int xdtype, int64_t N, int m, int64_t ldx, float* G, int64_t ldg,
              int accumulate, void* workspace, size_t workspace_bytes, void* stream);

/* A batch of Grams of one shape in ONE data-parallel launch: G[z] = X[z]ᵀX[z] for z < batch
 * (STORE), X: host array of `batch` device pointers to N x m fp16 / bf16 matrices (ld ldx), G:
 * batch x m x m fp32 packed.  256 x 256 tiles, every tile one chain over all N rows (no
 * stream-K pieces, no hand-offs, no workspace), so each G[z] is bit-identical to pt2q_gram on
 * X[z] alone.  Needs m % 256 == 0, ldx % 8 == 0, 16-byte aligned X[z] and batch <= 128, else
 * PT2Q_E_UNSUPPORTED (use pt2q_gram per item).  fp32 X (any m, batch <= 128): the f32 chain
 * GEMM over every item's upper tiles in one launch, again bit-identical per item.  Replaces
 * main.py:128 for every unit of a model step whose activations are at hand (the q/k/v, o,
 * gate/up inputs of all decoder layers). */
int pt2q_gram_batched(int batch, const void* const* X, int xdtype, int64_t N, int m, int64_t ldx,
                      float* G, void* stream);
/* pt2q_gram_batched (16-bit X only) storing ONLY the upper triangle of each G (G[z][r][c] for
 * c >= r; the strictly lower part is left as it was): a per-channel unit's Gram feeds nothing but
 * S1 / d (quantizer.py:215-218), which pt2q_s1_from_upper_batched forms from the upper triangle
 * with the same bits -- half the epilogue's stores.  PT2Q_E_UNSUPPORTED for fp32 X. */
int pt2q_gram_batched_upper(int batch, const void* const* X, int xdtype, int64_t N, int m, int64_t ldx,
                            float* G, void* stream);

/* H = G / nsamples; H_ii += percdamp * mean(diag H).  Replaces main.py:129-133 and
 * gptq.py:94-98.  damp_dev (nullable) receives the damping value. */
int pt2q_prepare_hessian(const float* G, int64_t ldg, int m, int64_t nsamples, float percdamp,
                         float* H, int64_t ldh, float* damp_dev, void* stream);

/* Hinv = cholesky_inverse(cholesky(H)) (main.py:136-139, gptq.py:101-103), full symmetric.
 * info_dev receives 0, or k+1 for the first non-positive pivot (then Hinv is undefined and the
 * caller applies torch.linalg.pinv, main.py:140-141). */
int pt2q_cholesky_inverse(const float* H, int64_t ldh, int m, float* Hinv, int64_t ldhi,
                          void* workspace, size_t workspace_bytes, int* info_dev, void* stream);

/* A batch of units' inverse Hessians in one launch sequence (main.py:129-139 for each unit of a
 * model step whose raw Grams are all at hand): for z < batch, H_z = G_z / nsamples + damping
 * (as pt2q_prepare_hessian), Hinv_z = cholesky_inverse(cholesky(H_z)).  G, H, Hinv are packed
 * batch x m x m fp32 (item z at + z*m*m); H is scratch and holds the factors U_z on return.  Every
 * step of the blocked factorisation serves all items in one launch (grid.y = item), so the
 * latency-bound diagonal and panel steps of small m fill the chip; each item's result is
 * bit-identical to pt2q_prepare_hessian + pt2q_cholesky_inverse on it alone.  info_dev: batch
 * ints (0, or k+1 at the first non-positive pivot; then that item falls back to pinv on the host,
 * main.py:140-141).  workspace: pt2q_hessian_inverse_batched_workspace_bytes(m, batch). */
size_t pt2q_hessian_inverse_batched_workspace_bytes(int m, int batch);
int pt2q_hessian_inverse_batched(const float* G, int m, int batch, int64_t nsamples, float percdamp,
                                 float* H, float* Hinv, void* workspace, size_t workspace_bytes,
                                 int* info_dev, void* stream);

/* The block loop of main.py:158-230 (flags & PT2Q_AGA_ACT) or gptq.py:124-199 (PT2Q_AGA_HESS).
 *   W      n x m weights (row-major, wdtype), read only.
 *   A      AGA matrix: raw Gram XᵀX (ACT) or damped H (HESS); m x m; may be NULL for NONE.
 *   Hinv   m x m inverse Hessian; read by the error feedback only, so it may be NULL when
 *          b >= m (one block: per-channel quantisation, main.py:198 never feeds back).
 *   alpha, mu  n x B fp32 (B = ceil(m/b)), column k = k-th selected block.
 *   T      n x m codes in ORIGINAL column order, int8 (tdtype PT2Q_I8) or fp32 (PT2Q_F32).
 *   perm   m int64, concatenated block indices in selection order.
 *   iters_dev  (nullable) B ints, ITF iterations per block. */
int pt2q_quantize_blocks(const void* W, int wdtype, int64_t ldw, int n, int m, int b, int flags,
                         const float* A, int64_t lda, const float* Hinv, int64_t ldhi,
                         int max_iter, float* alpha, float* mu, void* T, int tdtype,
                         int64_t* perm, int* iters_dev, void* workspace, size_t workspace_bytes,
                         void* stream);

/* The block loops of `count` (1..16) linears of one shape in ONE launch sequence: every block
 * step's selection, ATQ and error-feedback launches serve all of them (grid.z = linear), so the
 * latency-bound per-block kernels of small layers fill the chip and the error feedback's
 * persistent workgroups stream the tiles of every linear.  Linear z: weights W[z], AGA matrix
 * A[z] (raw Gram, PT2Q_AGA_ACT) and Hinv[z] (each m x m, leading dims lda / ldhi), outputs
 * alpha[z], mu[z], T[z], perm[z], iters_dev[z] (nullable array / entries) exactly as
 * pt2q_quantize_blocks on that linear alone -- bit for bit.  The pointer arrays are HOST arrays of
 * device pointers, read during the call only.  Supports blocks of <= 128 columns with b < m,
 * PT2Q_AGA_ACT or PT2Q_AGA_NONE, n <= 16384 with n % 4 == 0 (pt2q_quantize_blocks_group_supported); else PT2Q_E_UNSUPPORTED (use
 * pt2q_quantize_blocks per linear).  Replaces main.py:158-230 run over a list of linears (the
 * q/k/v of several decoder layers, main.py:289-299).  workspace:
 * pt2q_quantize_blocks_group_workspace_bytes(count, n, m, b, flags). */
size_t pt2q_quantize_blocks_group_workspace_bytes(int count, int n, int m, int b, int flags);
/* 1 if pt2q_quantize_blocks_group takes n x m linears with block b and these flags (every
 * condition of its PT2Q_E_UNSUPPORTED return, including the tuning overrides and the error
 * feedback's buffer limits: m % 4 == 0, m * round_up(n, 64) * 4 < 2 GiB), else 0. */
int pt2q_quantize_blocks_group_supported(int n, int m, int b, int flags);
int pt2q_quantize_blocks_group(int count, const void* const* W, int wdtype, int64_t ldw, int n, int m,
                               int b, int flags, const float* const* A, int64_t lda,
                               const float* const* Hinv, int64_t ldhi, int max_iter,
                               float* const* alpha, float* const* mu, void* const* T, int tdtype,
                               int64_t* const* perm, int* const* iters_dev, void* workspace,
                               size_t workspace_bytes, void* stream);

/* Per-channel block loops (b >= m > 512: one block of every column in ascending order,
 * main.py:158-230 with block_size >= in_features; BASELINE config 5) of `count` (1..16) linears
 * of one width m and W dtype in ONE launch sequence -- their row counts n[z] may differ (the
 * q/k/v/o and gate/up projections of a Llama layer share m).  A 5120-row linear alone fills 1.25
 * waves per SIMD; the group's rows share one grid.  Linear z: row-major W[z] (n[z] x m, leading
 * dim ldw), S1d[z] = S1 (m floats) then d -- a row of pt2q_s1_from_gram_batched (variant M, the
 * raw Gram's S·1 and 1ᵀS1, quantizer.py:215-218; a NULL array or entry = no AGA) -- outputs
 * alpha[z], mu[z] (n[z] fp32), T[z] (n[z] x m, tdtype, leading dim m), perm[z] (m int64: [0, m))
 * and iters_dev[z] (1 int; nullable array / entries), each exactly pt2q_quantize_blocks(W[z], ...,
 * b = m, PT2Q_FLAG_S1_GIVEN | PT2Q_AGA_ACT) -- bit for bit.  Pointer arrays are HOST arrays of
 * device pointers, read during the call only.  Replaces main.py:289-299's per-linear calls for a
 * list of per-channel linears.  workspace: pt2q_quantize_perchannel_group_workspace_bytes(count). */
size_t pt2q_quantize_perchannel_group_workspace_bytes(int count);
int pt2q_quantize_perchannel_group(int count, const void* const* W, int wdtype, int64_t ldw, const int* n,
                                   int m, const float* const* S1d, int max_iter, float* const* alpha,
                                   float* const* mu, void* const* T, int tdtype, int64_t* const* perm,
                                   int* const* iters_dev, void* workspace, size_t workspace_bytes,
                                   void* stream);

/* Whole layer, variant M (main.py:102-230): gram -> prepare -> cholesky_inverse -> blocks.
 * If info_dev reports a breakdown the outputs are undefined; the caller recomputes Hinv with
 * pinv and calls pt2q_quantize_blocks (the staged path). */
int pt2q_quantize_layer(const void* W, int wdtype, int64_t ldw, int n, int m, const void* X,
                        int xdtype, int64_t N, int64_t ldx, int b, int flags, float percdamp,
                        int max_iter, float* alpha, float* mu, void* T, int tdtype,
                        int64_t* perm, int* iters_dev, int* info_dev, void* workspace,
                        size_t workspace_bytes, void* stream);

/* One ATQ stage on W (n x b, row-major fp32, leading dim ldw) (quantizer.py:32-293).
 * alpha, mu: n fp32 (in for ROUND/ITF, out otherwise); T: n x b fp32, leading dim ldt
 * (in for GRID/ITF/AGA, out for INIT/ROUND/ITF/FULL); S1 (b) and d_dev (1) for AGA/FULL
 * (NULL S1 in FULL = no activations).  iters_dev (nullable) receives ITF iterations. */
int pt2q_atq_stage(int mode, const float* W, int64_t ldw, int n, int b, float* alpha, float* mu,
                   float* T, int64_t ldt, const float* S1, const float* d_dev, int max_iter,
                   int* iters_dev, void* workspace, size_t workspace_bytes, void* stream);

/* S1 = S·1 and d = 1ᵀS1 for a symmetric b x b matrix S (quantizer.py:215-218). */
int pt2q_s1_from_gram(const float* S, int64_t lds, int b, float* S1, float* d_dev, void* stream);
/* The same for `batch` whole m x m Grams (item z at S + z * item_stride, leading dim lds) in one
 * launch pair: S1d[z * (m + 1) + j] = S1[j] of item z, S1d[z * (m + 1) + m] = its d; bit-identical
 * to pt2q_s1_from_gram per item.  Per-channel quantisation (block_size >= m, quantizer.py:215-218
 * on the whole Gram) feeds S1d rows to pt2q_quantize_blocks with PT2Q_FLAG_S1_GIVEN, once per
 * Gram instead of once per linear (q/k/v and gate/up share one, main.py:289-299). */
int pt2q_s1_from_gram_batched(const float* S, int64_t lds, int m, int batch, int64_t item_stride, float* S1d,
                              void* stream);
/* pt2q_s1_from_gram_batched reading only the upper triangle of each S (S[c][r] for c < r taken
 * from S[r][c]: the Gram's mirror is an exact copy) -- bit-identical on a symmetric S, and valid
 * on pt2q_gram_batched_upper's output.  m > 512, m % 4 == 0, 16-byte aligned rows (else
 * PT2Q_E_UNSUPPORTED). */
int pt2q_s1_from_upper_batched(const float* S, int64_t lds, int m, int batch, int64_t item_stride, float* S1d,
                               void* stream);

/* compute_column_similarity_to_mean + select_next_block_ssr (reorder.py:36-61,107-143) on W
 * (n x m row-major fp32).  rem: r int64 ascending.  Writes min(b,r) entries of blk (selection
 * order), r - min(b,r) entries of newrem (ascending), and r similarities to sim (nullable;
 * untouched when r <= b). */
size_t pt2q_ssr_workspace_bytes(int n, int m);
int pt2q_ssr_select(const float* W, int64_t ldw, int n, int m, const int64_t* rem, int r, int b,
                    int64_t* blk, int64_t* newrem, float* sim, void* workspace,
                    size_t workspace_bytes, void* stream);

/* One block's GPTQ error feedback, in place (main.py:187-214, gptq.py:158-186):
 *   C = Hinv[blk][:, rem] / clamp(diag(Hinv)[blk], 1e-8);  W[:, rem] -= E @ C
 * W n x m fp32 row-major (updated), blk: bs int64, rem: r int64 (the columns still to quantise),
 * E: n x bs fp32 (the block's quantisation error W_b - (alpha*T + mu)), Hinv m x m.  The product
 * is rounded before the subtraction, as in the reference.  pt2q_quantize_blocks runs the same
 * kernels inside its loop. */
size_t pt2q_error_feedback_workspace_bytes(int n, int m, int bs);
int pt2q_error_feedback(float* W, int64_t ldw, int n, int m, const int64_t* blk, int bs,
                        const int64_t* rem, int r, const float* E, int64_t lde, const float* Hinv,
                        int64_t ldhi, void* workspace, size_t workspace_bytes, void* stream);

/* Reconstruct W_q[:, perm[kb:(k+1)b]] = alpha[:,k] * T + mu[:,k] (gptq.py:201-230). T int8 or
 * fp32 (tdtype), out fp32 n x m. */
int pt2q_dequantize(const float* alpha, const float* mu, const void* T, int tdtype,
                    const int64_t* perm, int n, int m, int b, float* out, void* stream);

/* 2-bit packing of ternary codes, utils.py:189-219 layout ({-1,0,1} -> {0,1,2}, 4 per byte,
 * little end first). count codes -> ceil(count/4) bytes. */
int pt2q_pack_ternary(const int8_t* T, int64_t count, uint8_t* packed, void* stream);
int pt2q_unpack_ternary(const uint8_t* packed, int64_t count, int8_t* T, void* stream);

/* out = ((parts[0] + parts[1]) + parts[2]) + ... + parts[nparts-1], elementwise fp32 in rank order;
 * part p starts at parts + p*stride (count floats each; count and stride multiples of 4, 16-byte
 * aligned; out may be parts[0]).  The deterministic reduction of the intra-layer split
 * (the Gram of main.py:128 data-parallel over the N calibration rows, one partial
 * Gram per rank, folded on the destination rank in rank order) -- an all-reduce would leave the
 * order to the ring schedule. */
int pt2q_sum_partials(const float* parts, int64_t stride, int nparts, int64_t count, float* out,
                      void* stream);

/* Counter-based synthetic tensors (tests/synth.py): out[i] = c_i * scale with
 * c_i = (splitmix64(splitmix64(seed) + i) >> 40) - 2^23; when outlier_every > 0, columns j
 * (= i % cols) with splitmix64(splitmix64(seed ^ 0x5BD1E995) + j) % outlier_every == 0 use
 * scale_outlier instead. fp32 out. */
int pt2q_fill_synthetic(float* out, int64_t count, uint64_t seed, float scale, int64_t cols,
                        int outlier_every, float scale_outlier, void* stream);

/* ---- Ternary inference (model.py:17-127 TernaryLinear) ----
 * y[t][i] = Σ_p Wd[i][p] x[t][g[p]] + bias[i], Wd[i][p] = xdtype(alpha[i][p/bs]·c[i][p] + mu[i][p/bs]).
 * Positions p are the input columns in block order (P = pt2q_ternary_linear_positions(m),
 * padded to 128).  pt2q_ternary_pack lays out the 2-bit codes (n x P/4 bytes) and the gather
 * index g (P int32) once per layer from the quantizer's outputs (T int8 n x m in ORIGINAL column
 * order, perm int64 m): mode 0 = correct reconstruction (gptq.py:201-230), mode 1 = the
 * reference TernaryLinear.forward exactly as written (its double permutation, model.py:75-95). */
size_t pt2q_ternary_linear_positions(int m);
int pt2q_ternary_pack(const int8_t* T, int64_t ldt, int n, int m, const int64_t* perm, int mode,
                      uint8_t* codes, int* gather, void* stream);
/* x: tokens x m (fp16 or bf16, leading dim ldx); alpha, mu: n x B fp32; bias: n fp32 or NULL;
 * y: tokens x n (ydtype = xdtype or PT2Q_F32). */
size_t pt2q_ternary_linear_workspace_bytes(int tokens, int n, int m);
int pt2q_ternary_linear(const void* x, int xdtype, int tokens, int64_t ldx, int n, int m,
                        const uint8_t* codes, const int* gather, const float* alpha,
                        const float* mu, int B, int bs, const float* bias, void* y, int ydtype,
                        int64_t ldy, void* workspace, size_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PT2Q_H */
