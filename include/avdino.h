/*
 * avdino.h -- C ABI of libavdino.so, the MI355X (gfx950) kernels of the multimodal-DINO
 * training step of wardvdnb/Multimodal-SSL-AVMNIST.
 *
 * The reference has no FFI: its hot path is Python over ATen.  Each
 * entry point below replaces the ATen op sequence named in its comment (paths relative to
 * the reference's AVMNIST_Experiments/).  The Python host package
 * (multimodal-ssl-avmnist_amd/avdino) binds this header through ctypes; INTEGRATION.md
 * shows the binding.
 *
 * Contract (all functions):
 *   - plain pointers + sizes; the caller owns every device buffer (including partial-sum
 *     workspaces, sized with the *_parts / *_chunks / *_rows helpers); the library allocates no
 *     device memory;
 *   - host-side state: per-process caches filled on first use and read-only afterwards -- the
 *     CU count and the occupancy of each persistent kernel (hipOccupancy queries that size the
 *     persistent grids, e.g. conv_ws.hip ws_occ, conv_c1p.hip, wgrad_ws.hip, conv3.hip, c1w3.hip,
 *     conv_ws8.hip); no environment variable is read; no state depends on the data, so calls
 *     are reentrant for distinct streams (the first calls race benignly: every thread computes
 *     the same value).  The one mutable setting is the avd_options test hook (avd_set_options):
 *     it must not change while launches are being issued, nor between a *_rows / *_parts /
 *     *_chunks sizing query and the launch whose buffer it sized (the row counts of the
 *     persistent kernels follow options.grid_cap);
 *   - `stream` is a hipStream_t (NULL = default stream); launches are asynchronous;
 *   - return AVD_OK (0) or a negative avd_status; shapes are validated before any launch;
 *   - layouts: conv feature maps are channels-last NHWC ([N, H, W, C], bf16 or f32), N = G*B
 *     samples stored group-major (group g = view g owns samples g*B .. g*B+B-1); a stack's last
 *     pooled map can also be written as the reference's (c, h, w) flatten [N, C*H*W] (f32) for
 *     the Linear that follows; dense-head tensors are row-major f32 [rows, features];
 *   - reductions are deterministic (fixed-order partial sums, no float atomics): the same
 *     inputs give bitwise-identical outputs run to run.
 *
 * SURVEY.md 8(b) sketched an `avd_tensor` descriptor ABI ({data, dtype, ndim, shape[5],
 * stride[5]}); this header passes plain pointers, dtype codes and the few sizes each kernel
 * needs instead -- every tensor on this path is dense, so strides carry no information, and a
 * ctypes / cgo / JNI binding of scalars is simpler than of a struct.  Leading dimensions appear
 * explicitly where a kernel reads or writes a strided slice (GEMM ld / offsets).
 */
#ifndef AVDINO_H
#define AVDINO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum { AVD_F32 = 0, AVD_BF16 = 1 } avd_dtype;

typedef enum {
  AVD_OK = 0,
  AVD_ERR_SHAPE = -1,       /* unsupported / inconsistent shape */
  AVD_ERR_DTYPE = -2,       /* unsupported dtype combination */
  AVD_ERR_HIP = -3,         /* a HIP launch failed (hipGetLastError) */
  AVD_ERR_ARG = -4          /* null pointer / bad enum */
} avd_status;

/* Library version, (major << 16) | minor. */
int avd_version(void);
/* Human-readable name of the last HIP error seen by this thread (or "ok"). */
const char* avd_last_error(void);

/* Launch options.  The library reads no environment variables: every kernel route is the
 * measured default unless a caller sets one of these test hooks explicitly (process-wide, set
 * between launches, not while kernels are being queued from another thread):
 *   grid_cap      > 0: the persistent kernels (conv_ws, wgrad_ws, conv_ws8, the conv1 passes)
 *                 launch at most this many blocks, so at test sizes every block walks several
 *                 tiles as at bench size; 0 = no cap;
 *   generic_conv  1: every bf16 mid-layer conv / input gradient / weight gradient on the generic
 *                 conv_cl / wgrad_cl kernels instead of the weights-stationary ones;
 *   generic_m2    1: the BN-backward reduce of a (c,h,w)-flatten tail on the generic pooled
 *                 reduce instead of its dedicated kernel. */
typedef struct {
  int grid_cap;
  int generic_conv;
  int generic_m2;
} avd_options;
/* Copy *opts into the library (NULL: the defaults, all zero). */
int avd_set_options(const avd_options* opts);
/* The current options. */
int avd_get_options(avd_options* opts);

/* ------------------------------------------------------------------ conv blocks
 * One CentralNet / CNN block is conv(KxK, stride 1) -> BatchNorm2d(train) -> ReLU -> maxpool2
 * (models/unimodal.py:127-153 and 185-211; models/dino.py:18-73).
 */

/* BatchNorm2d / BatchNorm1d train-mode statistics, per (group, channel):
 * parts [C, G, R, 2] f32 partial (sum, sumsq) rows, channel-major (R rows per group: for
 * conv stats R = B*T), count = elements per (group, channel).  Outputs mean/invstd/scale/shift [G,C] (scale = gamma*invstd,
 * shift = beta - mean*scale).  If running_mean != NULL, applies the reference's sequential
 * per-call update for g = 0..G-1: rm = 0.9 rm + 0.1 mean_g, rv = 0.9 rv + 0.1 var_g*n/(n-1)
 * (nn.BatchNorm momentum 0.1; group order = the reference's call order, dino.py:680-704).
 * parts is consumed: the chunked first pass writes f64 chunk sums over it.
 * pivot (nullable): the partials are sums of (x - K) and (x - K)^2 with K = pivot[g * pivot_gs + c]
 * (shifted sums: no cancellation in the variance when |mean| >> std).  pivot_gs = C for a
 * per-(group, channel) pivot [G,C] (avd_colstats), 0 for one pivot per channel [C] -- which may
 * be running_mean itself (avd_cl_conv_fwd_pv's pivot: read before the running update). */
int avd_bn_finalize(float* parts, int G, int R, int C, long long count,
                    const float* gamma, const float* beta, float eps, float momentum,
                    float* mean, float* invstd, float* scale, float* shift,
                    float* running_mean, float* running_var, const float* pivot, int pivot_gs,
                    void* stream);

/* From the partials [C, G, R, 2] build the input-gradient coefficients
 * coef [G, C, 3] (dy = k1*dz + kx*y + k0) and write dgamma/dbeta/dbias [C] (sums over
 * groups; dbias = sum of dy = the grad of a bias feeding this BN, NULL to skip).
 * accumulate != 0 adds into dgamma/dbeta/dbias instead of overwriting. */
int avd_bn_bwd_finalize(const float* parts, int G, int R, int C, long long count,
                        const float* gamma, const float* mean, const float* invstd,
                        float* coef, float* dgamma, float* dbeta, float* dbias, int accumulate,
                        void* stream);

/* ------------------------------------------------------------------ dense layers */

/* C[m,n] = alpha * sum_k A[m,k] B[k,n] + bias[n] + beta * C[m,n]   (f32 in HBM, any strides)
 * nn.Linear forward (x W^T + b), input grad (dy W) and weight grad (dy^T x).
 * mode 0: f32 VALU FMA; mode 1: f32 MFMA (v_mfma_f32_16x16x4_f32, exact f32 products);
 * mode 2: bf16 MFMA (operands rounded to bf16, f32 accumulate; the bf16 training mode).
 * Modes 1/2 split deep-K products (weight gradients, K = batch rows) across blocks when the
 * caller passes a workspace of avd_gemm_ws_elems(M,N,K,mode) floats: partial tiles are summed
 * in fixed split order by a second kernel (deterministic, no atomics; ws may be NULL, then
 * one pass over K).  Results do not depend on the workspace beyond that choice. */
long long avd_gemm_ws_elems(int M, int N, int K, int mode);
int avd_gemm(int M, int N, int K, const float* A, long long sam, long long sak,
             const float* B, long long sbk, long long sbn, float* C, long long ldc,
             const float* bias, float alpha, float beta, int mode, float* ws,
             long long ws_elems, void* stream);

/* nn.Linear backward's two GEMMs in ONE launch (modes 1/2): dW [O, In] = dout^T x and
 * dX [rows, In] = dout W (W [O, In]); dout [rows, O] (leading dimension dout_ld), x [rows, In]
 * (x_ld), dX leading dimension dx_ld.  Both read dout, neither depends on the other: their tile
 * grids run side by side (one launch boundary, and two small grids fill the chip together);
 * results are bitwise those of the two avd_gemm calls.  ws: avd_linear_bwd_ws_elems floats of
 * split-K scratch (NULL: single passes over K).  db (nullable) = the bias gradient
 * sum_r dout[r, :], formed by extra blocks of the same launches (row-chunk partials in ws, then
 * a fixed-order fold in the split-K reduce launch): deterministic, no separate reduction
 * launches; needs ws (AVD_ERR_ARG without it).  which: 3 = both gradients; 1 = dW (+ db) only,
 * 2 = dX only (x / dW or W / dX may then be NULL) -- the step runs dX on its critical stream and
 * dW beside it on another one (same results as which = 3). */
long long avd_linear_bwd_ws_elems(int rows, int O, int In, int mode);
int avd_linear_bwd(int rows, int O, int In, const float* dout, long long dout_ld, const float* x,
                   long long x_ld, const float* W, float* dW, float* dX, long long dx_ld, float* db,
                   int mode, int which, float* ws, long long ws_elems, void* stream);

/* The encoder Linear of CentralUnimodalImage / Audio (unimodal.py:153 fc: Linear(1600 / 3136, E)
 * over x.view(N, -1) of the last conv block's pooled map, dino.py:459-468) in the bf16 step, over
 * the pooled map as it lies in HBM: feat [rows][HW*C] bf16 NHWC, i.e. features in (h, w, c)
 * order, while W [O][C*HW] f32 keeps the reference's (c, h, w) flatten order (state_dict, Adam,
 * EMA, all-reduce unchanged).  bf16 MFMA, f32 accumulate -- the same products as avd_gemm mode 2
 * over the f32 (c, h, w) features, whose bf16 rounding the tail pass now does when it stores them.
 *   avd_linear_weight_hwc: n <= 4 weights per launch, Wp[e] [O][HW*C] bf16 = W[e] with its
 *     columns in (h, w, c) order (per step, after Adam / EMA changed W);
 *   avd_linear_fwd_hwc: out[r*out_ld + o] = sum_i feat[r][i] Wp[o][i] + bias[o] (f32);
 *   avd_linear_bwd_hwc: dW[o][(c,h,w)] = sum_r dout[r][o] feat[r][(h,w,c)] (f32, the reference's
 *     order), db[o] = sum_r dout[r][o] (nullable), dX[r][(h,w,c)] = sum_o dout[r][o] Wp[o][...]
 *     stored bf16 -- the last conv block's pooled gradient in NHWC (avd_cl_bn_bwd_* mode 0);
 *     one paired launch + its split-K reduces, as avd_linear_bwd (which: as there).
 * ws: avd_linear_hwc_ws_elems floats (required by the backward).  C*HW % 8 == 0, O % 4 == 0,
 * feat / Wp / dout 16-byte aligned. */
long long avd_linear_hwc_ws_elems(int rows, int O, int In);
int avd_linear_weight_hwc(int n, const float* const* W, void* const* Wp, const int* O, const int* C,
                          const int* HW, void* stream);
int avd_linear_fwd_hwc(int rows, int O, int C, int HW, const void* feat, const void* Wp,
                       const float* bias, float* out, long long out_ld, float* ws,
                       long long ws_elems, void* stream);
int avd_linear_bwd_hwc(int rows, int O, int C, int HW, const float* dout, long long dout_ld,
                       const void* feat, const void* Wp, float* dW, float* db, void* dX, int which,
                       float* ws, long long ws_elems, void* stream);

/* ------------------------------------------------------------------ channels-last conv blocks
 * The training path's conv blocks on NHWC maps ([N][H][W][C]; Cin = 1 maps are the plain
 * images), on MFMA for both storage types: dt = AVD_BF16 (v_mfma_f32_16x16x32_bf16) or AVD_F32
 * (v_mfma_f32_16x16x4f32, exact f32 products -- the parity mode).  They replace one
 * conv -> BatchNorm2d(train) -> ReLU -> max_pool2d(2) block of CentralUnimodalImage /
 * CentralUnimodalAudio.forward (unimodal.py:127-221) and the 3x3 CNN blocks (dino.py:18-73),
 * forward and backward.  K in {3, 5}; Cin = 1 or a multiple of 8; Cout a multiple of 8.
 *
 * Weights: wk = avd_cl_weight_layout(w [Cout,Cin,K,K] f32) in dt, dgrad=0 for the forward,
 * dgrad=1 (flipped taps, swapped channels) for the input gradient; avd_cl_weight_elems gives
 * its element count. */
int avd_cl_weight_elems(int Cout, int Cin, int K, int dgrad);
int avd_cl_weight_layout(const float* w, void* wk, int dt, int Cout, int Cin, int K, int dgrad,
                         void* stream);
/* n <= 16 layouts in one launch (a conv stack's per-step weights): HOST arrays of n entries,
 * entry e = avd_cl_weight_layout(w[e], wk[e], dt, cout[e], cin[e], k[e], dgrad[e]). */
int avd_cl_weight_layout_batch(int n, const float* const* w, void* const* wk, const int* cout,
                               const int* cin, const int* k, const int* dgrad, int dt,
                               void* stream);

/* y = conv2d(x, w) + bias (stride 1, zero padding pad), x [N,H,W,Cin] -> y [N,Ho,Wo,Cout].
 * stats != NULL: BatchNorm partial (sum, sumsq) of the stored y values, [Cout][G][R][2] with
 * G = N/B groups (B = samples per BN group = per view) and R = avd_cl_stat_rows(...) rows per
 * group, for avd_bn_finalize. */
int avd_cl_stat_rows(int Ho, int Wo, int B, int K, int Cin, int Cout, int dt);
int avd_cl_conv_fwd(const void* x, const void* wk, const float* bias, void* y, float* stats,
                    int dt, int N, int B, int Cin, int H, int W, int Cout, int K, int pad,
                    void* stream);
/* 1 if the statistics producer of this shape takes a pivot (the persistent weights-stationary
 * mid layers, whose lane-local running sums span thousands of values per BN group). */
int avd_cl_stat_pivot(int Ho, int Wo, int B, int K, int Cin, int Cout, int dt);
/* avd_cl_conv_fwd with statistics about a per-channel pivot [Cout] (nullable; only where
 * avd_cl_stat_pivot, else AVD_ERR_ARG): the partials are sums of (y - pivot[c]) and
 * (y - pivot[c])^2 -- finalize with avd_bn_finalize(..., pivot, pivot_gs = 0).  The engine
 * passes the layer's BatchNorm running mean: near every batch's mean once it has tracked a few
 * batches, so the variance keeps full precision when |mean| >> std. */
int avd_cl_conv_fwd_pv(const void* x, const void* wk, const float* bias, const float* pivot,
                       void* y, float* stats, int dt, int N, int B, int Cin, int H, int W, int Cout,
                       int K, int pad, void* stream);

/* dx [N,H,W,Cin] = input gradient of the conv for dy [N,Ho,Wo,Cout]; wk_d = dgrad layout. */
int avd_cl_conv_dgrad(const void* dy, const void* wk_d, void* dx, int dt, int N, int Cin, int H,
                      int W, int Cout, int K, int pad, void* stream);

/* dw_parts[c] [Cout][Cin][K][K] f32 = weight gradient over sample chunk c of
 * avd_cl_wgrad_chunks(...) chunks; reduce with avd_sum_rows (fixed order). */
int avd_cl_wgrad_chunks(int N, int Cout, int Cin, int K);
int avd_cl_conv_wgrad(const void* x, const void* dy, int dt, float* dw_parts, int N, int Cin,
                      int H, int W, int Cout, int K, int pad, void* stream);

/* out = maxpool2(relu(y*scale[g,c] + shift[g,c])) over NHWC y (floor mode, first-max ties):
 *   mode 0: out NHWC [N,H/2,W/2,C] in dt;  mode 1: global average of that, f32 [N,C];
 *   mode 2: f32 [N, C*(H/2)*(W/2)] flattened in (c, h, w) order (the encoder Linear input). */
int avd_cl_bn_relu_pool(const void* y, int dt, const float* scale, const float* shift, void* out,
                        int mode, int N, int B, int C, int H, int W, void* stream);

/* Backward of the block above, given gout (mode 0: NHWC dt; mode 1: [N,C] f32; mode 2: f32 in
 * the mode-2 layout).  reduce: parts [C][G][R][2], R = avd_cl_bn_bwd_rows(...), then
 * avd_bn_bwd_finalize -> coef; apply: dy [N,H,W,C] (dt) = k1*dz + kx*y + k0. */
int avd_cl_bn_bwd_rows(int B, int C, int H, int W, int dt);
int avd_cl_bn_bwd_reduce(const void* y, int dt, const void* gout, int mode, const float* scale,
                         const float* shift, const float* mean, const float* invstd, float* parts,
                         int N, int B, int C, int H, int W, void* stream);
int avd_cl_bn_bwd_apply(const void* y, int dt, const void* gout, int mode, const float* scale,
                        const float* shift, const float* coef, void* dy, int N, int B, int C,
                        int H, int W, void* stream);

/* Fused BatchNorm-backward apply + conv weight gradient of a first (Cin = 1) layer whose output
 * is pooled in mode 0 -- the CentralNet audio conv1 (Cout 8, 5x5, pad 2, H, W % 16 == 0,
 * W <= 112) and the first 3x3 layer of the SimCLR / unimodal encoders (Cout 16/32, 3x3, pad 1,
 * H % 4 == 0, W even; models/dino.py:18-73), bf16: computes dy exactly as
 * avd_cl_bn_bwd_apply and, without storing it,
 * parts[s][Cout*K*K] = per-slab partial dW (reduce with avd_sum_rows over
 * avd_cl_apply_wgrad_slabs() rows).  Replaces avd_cl_bn_bwd_apply + avd_cl_conv_wgrad for that
 * layer (CentralUnimodalAudio.conv1/bn1, unimodal.py:160-190); the first layer needs no dx.
 * Returns AVD_ERR_SHAPE for any other shape (avd_cl_apply_wgrad_slabs() == 0). */
int avd_cl_apply_wgrad_slabs(int dt, int N, int Cin, int H, int W, int Cout, int K, int pad);
int avd_cl_bn_bwd_apply_wgrad(const void* y, const void* gout, const float* scale,
                              const float* shift, const float* coef, const void* x, float* parts,
                              int dt, int N, int B, int Cin, int H, int W, int Cout, int K, int pad,
                              void* stream);

/* Fused softmax cross-entropy over S = inv_t Q K^T without storing S (xent.hip): the InfoNCE
 * (dino.py:1091-1128) and NT-Xent (multimodal_simclr.py:74-89) losses with both gradients, for
 * this rank's rows q [R][P] (L2-normalised, f32) against the gathered columns k [C][P], on the
 * bf16 MFMA (flash-style: online row softmax, column pass from the row lse).  Row i is in half
 * h = i / Bh (R <= 2 Bh) with i' = i - h Bh; its target column is tgt_h + i', its masked column
 * msk_h + i' (msk_h < 0: none).  Writes loss[R] = lse_i - S[i][t(i)] (the unscaled per-row CE,
 * as avd_softmax_xent's loss_parts), dq[R][P] = gscale inv_t (sum_j p_ij k_j - k_t(i)) and
 * dk[C][P] = gscale inv_t (sum_i p_ij q_i - sum_{t(i) = j} q_i).  P = 128 or 256; ws holds
 * avd_xent_fused_ws(R, C, P) floats.  Deterministic (fixed-order partial sums, no atomics). */
int avd_xent_fused_ws(int R, int C, int P);
int avd_xent_fused(const float* q, const float* k, int R, int C, int P, int Bh, int tgt0, int tgt1,
                   int msk0, int msk1, float inv_t, float gscale, float* loss, float* dq, float* dk,
                   float* ws, long long ws_elems, void* stream);

/* Test hook: fill the LDS of every CU with NaN bit patterns (0x7fc07fc0), so a kernel that reads
 * LDS it never wrote sees NaN instead of a benign leftover (tools/lds_poison.py). */
int avd_lds_poison(void* stream);

/* The whole backward of the audio conv2 layer in one launch (lbwd.hip; CentralUnimodalAudio
 * conv2 -> bn2 -> ReLU -> MaxPool2d, unimodal.py:185-221: 56x56, Cin 8 -> Cout 16, 5x5 pad 2,
 * bf16): from y [N][56][56][16] and the pooled gradient gout [N][28][28][16] (layout 0) with
 * avd_bn_finalize's scale / shift and avd_bn_bwd_finalize's coef -- or, with y == NULL, from a
 * given dy -- it forms dy exactly as avd_cl_bn_bwd_apply (never stored), and from each staged dy
 * tile both
 *   dx [N][56][56][8]   = the input gradient, bit-identical to avd_cl_conv_dgrad (wk_d: the
 *                         avd_cl_weight_layout(..., dgrad = 1) rows), and
 *   parts[s][16*8*25]   = per-slab partial dW (sum with avd_sum_rows over `slabs` rows).
 * Replaces avd_cl_bn_bwd_apply + avd_cl_conv_dgrad + avd_cl_conv_wgrad for that layer.  `slabs`
 * is the grid: pass the avd_cl_layer_bwd_slabs() value the parts buffer was sized with (0: the
 * shape is not served).  N / B <= 8 BN groups when y is given. */
int avd_cl_layer_bwd_slabs(int dt, int N, int Cin, int H, int W, int Cout, int K, int pad);
int avd_cl_layer_bwd(const void* y, const void* gout, const float* scale, const float* shift,
                     const float* coef, const void* dy, const void* x, const void* wk_d, void* dx,
                     float* parts, int slabs, int dt, int N, int B, int Cin, int H, int W, int Cout,
                     int K, int pad, void* stream);

/* The partial sums of avd_cl_bn_bwd_reduce (same rows and layout, for avd_bn_bwd_finalize)
 * from the POOLED output p = maxpool2(relu(y*scale + shift)) instead of y: at the window's
 * argmax z = gamma*xhat + beta = p, so xhat = (p - beta)/gamma wherever the gradient is routed
 * (p > 0).  pooled has gout's layout (mode 0: NHWC dt = the next conv's input; mode 2: f32
 * (c,h,w) flatten = the encoder Linear's input); y is read only for channels with gamma == 0.
 * Reads 2/4 of y's bytes instead of 5/4.  Modes 0 and 2, even H and W. */
int avd_cl_bn_bwd_reduce_pooled(const void* y, int dt, const void* pooled, const void* gout,
                                int mode, const float* gamma, const float* beta, const float* mean,
                                const float* invstd, float* parts, int N, int B, int C, int H,
                                int W, void* stream);

/* The same first layer WITHOUT storing its conv output: every pass recomputes y = conv(x) + b
 * (bf16-rounded, bit-identical across passes) into an on-chip tile from the 8x smaller input.
 *   pass 0 (stats):  out = BN partial rows [Cout][G][R][2] of the rounded y
 *                    (R = avd_cl_c1_recompute_rows(0, ...); feed avd_bn_finalize); for the
 *                    3x3 1 -> 32 layer at 28^2 / 112^2 the rows are of the EXACT conv
 *                    output, formed from per-block patch Gram matrices (c1s3.hip);
 *   pass 1 (apply):  z = maxpool2(relu(y*scale + shift)) NHWC [N][H/2][W/2][Cout] (bf16);
 *   pass 2 (reduce): out = BN-backward partial rows (sum dz, sum dz*xhat) as
 *                    avd_cl_bn_bwd_reduce (mode 0), gz = pooled gradient;
 *   pass 3 (wgrad):  out = dW partial slabs as avd_cl_bn_bwd_apply_wgrad.
 *   pass 4 (reduce + weight-gradient moments in one pass): out = pass 2's rows
 *                    [Cout][G][R][2], then [R][G][avd_cl_c1_moment_cols(Cout, K)] moments:
 *                    Cout 16/32/64 (c1w3.hip): sum dz xk per channel/tap [Cout][KK], Gram rows of
 *                    the im2col xk with a ones tap [KK][KK+1] (KK = 9 for 3x3 pad 1, 25 for 5x5
 *                    pad 2 -- the CentralNet image conv1); the 5x5 audio conv1 (Cout 8): sum dz x25
 *                    [8][25], the x25 Gram matrix [25][25], sum x25 [25] (850).  dW is linear in
 *                    dy = k1 dz + kx y + k0, so after avd_bn_bwd_finalize and avd_sum_rows of
 *                    the moments, avd_cl_c1_recompute_combine forms dW (y taken unrounded).
 * scale/shift/mean/invstd [G][Cout] from avd_bn_finalize, coef from avd_bn_bwd_finalize.
 * Shapes: Cin 1, bf16, the 5x5 pad-2 1->8 audio conv1 at 112^2 (CentralUnimodalAudio conv1+bn1+
 * pool, unimodal.py:160-190), and 1->16/32/64 3x3 pad 1 or 5x5 pad 2 with W % 4 == 0, W <= 128
 * (the 3x3 encoders' first layers, dino.py:18-73; CentralUnimodalImage conv1+bn1+pool,
 * unimodal.py:127-141); rows() == 0 otherwise. */
int avd_cl_c1_recompute_rows(int pass, int dt, int N, int B, int Cin, int H, int W, int Cout,
                             int K, int pad);
int avd_cl_c1_recompute(int pass, const void* x, const void* wk, const float* bias,
                        const float* scale, const float* shift, const float* mean,
                        const float* invstd, const float* coef, const void* gz, void* z,
                        float* out, int dt, int N, int B, int Cin, int H, int W, int Cout, int K,
                        int pad, void* stream);
/* dW [Cout][1][K][K] = sum_g k1 M_dz + kx (w . Gram + b sum x) + k0 sum x from pass 4's
 * row-summed moments [G][avd_cl_c1_moment_cols(Cout, K)] and coef [G][Cout][3] (float64);
 * wk = the forward layout.  Cout 8: the 5x5 audio conv1; Cout 16/32/64: the 3x3 / 5x5 first
 * layers. */
int avd_cl_c1_moment_cols(int Cout, int K);
int avd_cl_c1_recompute_combine(const float* moments, const float* coef, const void* wk,
                                const float* bias, float* dw, int G, int Cout, int K, void* stream);

/* out[c] (+)= sum_{r<rows} in[r*ld + c]   (fixed order, f64 accumulation) -- reduces the conv
 * weight-grad partial slabs and gives Linear bias gradients (column sums of dy). */
int avd_sum_rows(const float* in, int rows, int cols, long long ld, float* out, int accumulate,
                 void* stream);

/* The same sum in two passes for tall, narrow inputs (Linear bias gradients over thousands of
 * rows, conv weight-grad slabs): avd_sum_rows_chunks(rows, cols) row chunks are summed in
 * parallel into work[chunk][cols] (work_elems >= chunks*cols), then reduced in chunk order.
 * chunks depends on the shape only (deterministic everywhere); 1 = single pass, work unused. */
int avd_sum_rows_chunks(int rows, int cols);
int avd_sum_rows_split(const float* in, int rows, int cols, long long ld, float* out,
                       int accumulate, float* work, long long work_elems, void* stream);

/* Column partial statistics of x [rows, C] f32 for BatchNorm1d: parts [C, G, R, 2] with
 * R = avd_colstats_parts(rows/G) row-chunks per group.  pivot [G,C] (nullable) receives
 * the first row of each group; the partials are then taken about it (pass it on to
 * avd_bn_finalize). */
int avd_colstats_parts(int rows_per_group);
int avd_colstats(const float* x, int rows, int G, int C, float* parts, float* pivot,
                 void* stream);

/* Elementwise activation with optional dropout (keep mask from a counter hash of
 * (seed, index), scaled by 1/(1-p)); act 0 = ReLU (fusion, dino.py:222-227),
 * act 1 = GELU(erf) after BN1d (ProjectionHead, dino.py:1243-1249; scale/shift [G,C]
 * per-column affine applied first, rows grouped into G groups of rows/G).
 * x [rows, C] f32 -> out [rows, C] f32. */
int avd_act_fwd(const float* x, float* out, int act, const float* scale, const float* shift,
                int rows, int G, int C, float p, unsigned long long seed, void* stream);

/* Backward of avd_act_fwd w.r.t. its input x (pre-affine value for act 1: returns dz, the
 * grad w.r.t. the BN output).  dout [rows,C] -> dx [rows,C]. */
int avd_act_bwd(const float* x, const float* dout, float* dx, int act, const float* scale,
                const float* shift, int rows, int G, int C, float p, unsigned long long seed,
                void* stream);

/* The same with the dropout seed offset by *seed_off (device memory; the step state of
 * avd_step_begin), so a captured step (hipGraph) draws fresh masks on every replay. */
int avd_act_fwd_dev(const float* x, float* out, int act, const float* scale, const float* shift,
                    int rows, int G, int C, float p, unsigned long long seed,
                    const unsigned long long* seed_off, void* stream);
int avd_act_bwd_dev(const float* x, const float* dout, float* dx, int act, const float* scale,
                    const float* shift, int rows, int G, int C, float p, unsigned long long seed,
                    const unsigned long long* seed_off, void* stream);

/* BatchNorm1d backward partials: parts [C, G, R, 2] = (sum dz, sum dz*xhat) per row chunk. */
int avd_bn1d_bwd_reduce(const float* x, const float* dz, const float* mean, const float* invstd,
                        int rows, int G, int C, float* parts, void* stream);

/* avd_act_bwd_dev (act 1: GELU over the BatchNorm1d affine, then dropout) and
 * avd_bn1d_bwd_reduce in one launch: dz = dropout(dout) * gelu'(scale*x + shift) is written to
 * dz and its partials (sum dz, sum dz*xhat) to parts [C, G, R, 2] -- bit-identical to the two
 * launches (same operations, same row order).  ProjectionHead backward, dino.py:1240-1254. */
int avd_bn1d_act_bwd_reduce(const float* x, const float* dout, float* dz, const float* scale,
                            const float* shift, const float* mean, const float* invstd, int rows,
                            int G, int C, float p, unsigned long long seed,
                            const unsigned long long* seed_off, float* parts, void* stream);

/* dx = k1*dz + kx*x + k0 per (group, column), coef [G,C,3] from avd_bn_bwd_finalize. */
int avd_bn1d_bwd_apply(const float* x, const float* dz, const float* coef, float* dx,
                       int rows, int G, int C, void* stream);

/* ------------------------------------------------------------------ losses */

/* DINO loss forward+backward (MultiModalDINOLightning.dino_loss, dino.py:822-854, plus the
 * centring of MultiModalDINO.forward, dino.py:709-720):
 *   t_raw [T*B, P] teacher projections (uncentred), center [P];
 *   s [V*B, P] student projections (view-major rows);
 *   loss_parts [V*B] per-row loss terms (sum = loss), ds [V*B, P] = d loss / d s;
 *   center_new [P] = m*center + (1-m)*mean_rows(t_raw)  (update_center, dino.py:648-653);
 *   center_teacher != 0: also subtract the per-view batch mean of the normalised teacher
 *   (UniModalDINOLightning.dino_loss, dino.py:1613-1614).
 *   work: >= (B + T*B) * P floats. */
int avd_dino_loss(const float* s, const float* t_raw, const float* center, int V, int T, int B,
                  int P, float tau_s, float tau_t, float center_m, int center_teacher,
                  float* loss_parts, float* ds, float* center_new, float* work, void* stream);

/* MSE between L2-normalised rows (MultiModalDINOWithMSELightning.mse_loss, dino.py:1193-1211):
 * a, b [B,P] -> loss_parts [B], da, db [B,P]. */
int avd_mse_loss(const float* a, const float* b, int B, int P, float* loss_parts,
                 float* da, float* db, void* stream);

/* Row-wise L2 normalisation (F.normalize, eps 1e-12): y = x / max(|x|, eps), norms [rows]. */
int avd_l2norm_fwd(const float* x, float* y, float* norms, int rows, int P, void* stream);
/* dx = (dy - y (y.dy)) / max(|x|, eps)  (dy overwritten-safe: dx may alias dy). */
int avd_l2norm_bwd(const float* y, const float* norms, const float* dy, float* dx, int rows,
                   int P, void* stream);

/* Softmax cross-entropy over rows of logits [R, C] (F.cross_entropy, dino.py:1001-1025 /
 * 1091-1128, multimodal_simclr.py:74-89): loss_parts [R] (unnormalised per-row -log p_target),
 * dlogits [R,C] = (softmax - onehot)*gscale (added to dlogits when accumulate != 0).
 * Targets: target_mode 0 = targets[r] (int64); 1 = r + tgt_off (InfoNCE diagonal, tgt_off =
 * this shard's first global row when the columns are all-gathered negatives); 2 = (r + R/2) % R
 * (NT-Xent positives over a local [2B] batch).  mask_off >= 0 excludes column r + mask_off
 * (NT-Xent self-similarity, multimodal_simclr.py:79-81); < 0 masks nothing.  col_major != 0
 * reads logits transposed (logits^T rows). */
int avd_softmax_xent(const float* logits, long long ld, int R, int C, const int64_t* targets,
                     int target_mode, int tgt_off, int col_major, int mask_off, float gscale,
                     float* loss_parts, float* dlogits, long long ldd, int accumulate,
                     void* stream);

/* correct[r] = 1.0f if argmax_j logits[r*ld + j] (first maximum, as torch.max) == targets[r],
 * else 0.0f -- the probe accuracy of evaluate() (dino.py:913-947). */
int avd_argmax_correct(const float* logits, long long ld, int R, int C, const int64_t* targets,
                       float* correct, void* stream);

/* Cosine-consistency term of the unimodal DINO loss (UniModalDINOLightning.
 * _cosine_consistency_loss, dino.py:1575-1594) over view-major embeddings emb [V*B, D]:
 * loss_parts [B] = alpha * per-sample share of mean_{i<j} mean_b (1 - n_i.n_j)^2 with
 * n = F.normalize(emb); demb [V*B, D] += alpha * d loss / d emb.  Either output may be NULL
 * (not both).  2 <= V <= 32. */
int avd_cosine_consistency(const float* emb, int V, int B, int D, float alpha, float* loss_parts,
                           float* demb, void* stream);

/* ------------------------------------------------------------------ input staging */

/* Re-lay a collated batch view-major for the encoder (MultiModalDINO.forward's per-view loop,
 * dino.py:680-704): out[(v*B + b)] = g[b, v] (v < G), then l[b, v-G] (v < G+L), then orig[b]
 * (if orig != NULL).  g [B,G,HW], l [B,L,HW], orig [B,HW] f32; out [(G+L+1?)*B, HW] (odt).
 * HW % 4 == 0. */
int avd_stage_views(const float* g, int G, const float* l, int L, const float* orig, int B,
                    int HW, void* out, int odt, void* stream);

/* ------------------------------------------------------------------ data path */

/* Device-side view augmentation: replaces the per-sample CPU transform chains of
 * MultiModalAugmentation.__call__ (utils/get_data.py:233-257; chains at 122-193).  One record
 * of AVD_AUG_REC floats per (sample b, view v) holds the already-drawn random parameters (the
 * host samples them, avdino/augment.py); the kernel applies, in the reference's order,
 *   RandomResizedCrop (bilinear, edge-clamped; the crops only up-sample, so antialias is a
 *   no-op) -> TimeWarpWithStretch (get_data.py:29-58: |phase_vocoder| = linear interpolation
 *   of magnitudes at t*rate, zero beyond) -> Frequency/TimeMasking (zero bands) ->
 *   RandomRotation -> RandomAffine (nearest, zero fill, torchvision's centred inverse matrix)
 *   -> RandomErasing (zero box) -> GaussianNoise (get_data.py:21-27; counter-hash normals) ->
 *   GroupedMasking (get_data.py:60-108; 4x4 groups, bitmask row gm[rec[AVD_AUG_GM]]).
 * src_u8 [N, H*W] raw dataset pixels, idx [B] int64 rows of src (the batch's sample ids),
 * lut [256] f32 = the dataset's normalisation of each byte value (get_data.py:464-467),
 * rec [B*V, AVD_AUG_REC], gm [*, gm_words] u32.  out f32: order 0 -> [B, V, H, W] (the
 * reference's collated views), order 1 -> [V, B, H, W] (view-major, the engine's layout). */
#define AVD_AUG_REC 28
enum {
  AVD_AUG_CROP = 0,    /* 0..3: top, left, h, w of the crop box */
  AVD_AUG_AFF = 4,     /* 4..9: RandomAffine inverse [m0 m1 m2; m3 m4 m5], centred coords */
  AVD_AUG_ROT = 10,    /* 10..15: RandomRotation inverse, same form */
  AVD_AUG_RATE = 16,   /* time-stretch rate */
  AVD_AUG_FMASK = 17,  /* 17,18: rows [f0, f1) zeroed */
  AVD_AUG_TMASK = 19,  /* 19,20: cols [t0, t1) zeroed */
  AVD_AUG_NOISE = 21,  /* gaussian noise std (0: none) */
  AVD_AUG_GM = 22,     /* grouped-mask bitmask row, < 0: none */
  AVD_AUG_FLAGS = 23,  /* bit 0 crop, 1 affine, 2 rotation, 3 time stretch */
  AVD_AUG_ERASE = 24   /* 24..27: top, left, h, w of the erased box (h = 0: none) */
};
int avd_augment_views(const uint8_t* src_u8, const int64_t* idx, long long n_src, int B, int V,
                      int H, int W, const float* lut, const float* rec, const uint32_t* gm,
                      int gm_words, int group, unsigned long long seed, int order, float* out,
                      void* stream);
/* The same with out in odt (AVD_F32 or AVD_BF16): with order 1 and bf16 the views land
 * straight in the engine's staged view-major input (no f32 round trip through
 * avd_stage_views). */
int avd_augment_views_dt(const uint8_t* src_u8, const int64_t* idx, long long n_src, int B,
                         int V, int H, int W, const float* lut, const float* rec,
                         const uint32_t* gm, int gm_words, int group, unsigned long long seed,
                         int order, void* out, int odt, void* stream);
/* Diagnostic (tools/dbg_prefetch6.py): the gather kernel into a bf16 out, and afterwards each block
 * re-checks its staged source row and byte table in LDS against global memory; chk[3] int32 on the
 * device: {LDS words found changed (accumulated), first changed word, its block}; seen
 * [B*V, AVD_AUG_REC] f32: the record fields each block used, as it read them. */
int avd_augment_views_lds_check(const uint8_t* src_u8, const int64_t* idx, int B, int V, int H, int W,
                                const float* lut, const float* rec, const uint32_t* gm, int gm_words,
                                int group, unsigned long long seed, int order, void* out, int* chk,
                                float* seen, void* stream);
/* Diagnostic: the gather kernel with its source row and byte table read from global memory, no
 * LDS staging (bf16 out). */
int avd_augment_views_nolds(const uint8_t* src_u8, const int64_t* idx, int B, int V, int H, int W,
                            const float* lut, const float* rec, const uint32_t* gm, int gm_words,
                            int group, unsigned long long seed, int order, void* out, void* stream);

/* The same views for a chain in ANY stage order (transforms.Compose order; the reference's own
 * configs/config_multimodal_dino.yaml best_augments chains, get_data.py:195-231, put the masks
 * and noise before the time stretch and the crop): kinds is a HOST array [nkinds <= 9] of
 * stage kinds in application order (the avd_augment_records numbering below); each applied
 * stage reads the previous stage's whole view (held in LDS), as each transform module reads its
 * predecessor's output.  A chain in the avd_augment_views order gives bit-identical views. */
int avd_augment_views_seq(const uint8_t* src_u8, const int64_t* idx, long long n_src, int B,
                          int V, int H, int W, const float* lut, const float* rec,
                          const uint32_t* gm, int gm_words, int group, unsigned long long seed,
                          int order, const int* kinds, int nkinds, void* out, int odt,
                          void* stream);

/* The records' random parameters drawn on the device (the get_params rules of each transform:
 * RandomResizedCrop / RandomErasing 10 attempts + fallback, RandomRotation / RandomAffine
 * inverse matrices, torchaudio mask_along_axis bands, time-stretch rate, noise std,
 * GroupedMasking's randperm(ng)[:k] as a uniformly random k-subset by Floyd's algorithm; one
 * thread per record).  stages is a HOST array [nstages <= 9][8] of {kind, p, params...}:
 *   kind 0 crop {scale0, scale1, ratio0, ratio1}, 1 time stretch {min, max},
 *   2 frequency mask {param}, 3 time mask {param}, 4 rotation {degrees},
 *   5 affine {degrees, translate_x (< 0: none), translate_y, scale0 (<= 0: none), scale1},
 *   6 erasing {scale0, scale1, ratio0, ratio1}, 7 gaussian noise {std},
 *   8 grouped masking {mask_ratio} (group size = group);
 * each stage draws U < p (applied) first, as RandomApply.  rec [n, AVD_AUG_REC] (record r's
 * grouped-mask row is r), gm [n, gm_words] (NULL without grouped masking; ng <= 1024). */
int avd_augment_records(const float* stages, int nstages, int n, int H, int W, int group,
                        unsigned long long seed, float* rec, uint32_t* gm, int gm_words,
                        void* stream);

/* ------------------------------------------------------------------ optimiser / EMA */

/* teacher = m*teacher + (1-m)*student over n floats (MultiModalDINO.update_teacher,
 * dino.py:635-646, on a flat parameter arena). */
int avd_ema(float* teacher, const float* student, long long n, float m, void* stream);

/* torch.optim.Adam step with L2 weight decay added to the gradient (configure_optimizers,
 * dino.py:953-962) over flat arenas p/g/m/v of n floats; bc1 = 1-b1^t, bc2 = 1-b2^t. */
int avd_adam(float* p, const float* g, float* m, float* v, long long n, float lr, float b1,
             float b2, float eps, float wd, float bc1, float bc2, void* stream);

/* torch.optim.AdamW step (decoupled weight decay: p *= 1 - lr*wd, then Adam without wd) --
 * the optimiser of the epoch-end linear probe (on_train_epoch_end, dino.py:898, 1678). */
int avd_adamw(float* p, const float* g, float* m, float* v, long long n, float lr, float b1,
              float b2, float eps, float wd, float bc1, float bc2, void* stream);

/* Device step state of a graph-replayable training step (the engine's per-step scalars live
 * in device memory, so one captured hipGraph replays every step):
 *   t        [1] int64 -- optimizer steps taken; avd_step_begin increments it,
 *   hyp      [4] f32   -- {lr (written by the host when the schedule moves), 1-b1^t, 1-b2^t, -}
 *                         (bias corrections in double, rounded once, as the host computes them),
 *   seed_off [1] u64   -- t_before * seed_stride, the dropout counter offset of this step
 *                         (may be NULL).
 * avd_adam_dev / avd_adamw_dev read lr and the bias corrections from hyp. */
/* arena[idx[i]] += val[i] for i < n, int64, distinct indices: the num_batches_tracked
 * increments of one forward for every BatchNorm layer at once (nn.BatchNorm*d.forward in
 * training mode, num_batches_tracked += 1 per call; dino.py:680-704 calls each layer per view). */
/* ---- the audio conv1 backward routed by forward codes (conv_c1p.hip; CentralUnimodalAudio conv1
 * -> bn1 -> relu -> maxpool, unimodal.py:185-190, 5x5 1->8 on 112x112, bf16).
 * avd_cl_c1_apply_codes = avd_cl_c1_recompute pass 1 (BN -> ReLU -> 2x2 max-pool z from the
 * recomputed y) that also writes codes [N][H/2][W/2] u32: nibble c (bits 4c..4c+3) = 1 + the
 * first argmax of relu(bn(y)) over the window when that max is > 0, else 0 -- the max-pool
 * indices of nn.MaxPool2d (first maximum) with ReLU's zero gradient folded in.
 * avd_cl_c1_moments_codes: ONE pass over x, the pooled gradient gz [N][H/2][W/2][8] and the
 * codes -> per (row r, group g) of avd_cl_c1_codes_rows rows: MOMC = avd_cl_c1_codes_cols()
 * floats: M[8][25] = sum dz x25 | Gram[25][25] = sum x25 x25^T | S[25] = sum x25 | sum dz [8],
 * out[(r * G + g) * MOMC + ...]; reduce the rows with avd_sum_rows.
 * avd_cl_c1_codes_combine (one launch, float64): the BN backward of bn1 (dgamma, dbeta, coef
 * [G][8][3] as avd_bn_bwd_finalize; sum dz y = w . M + b sum dz at the exact conv output), the
 * conv bias gradient dbias (= sum dy) and dW [8][25] = sum_g k1 M + kx (w Gram + b S) + k0 S.
 * count = B*H*W; coef / dgamma / dbeta / dbias nullable. */
int avd_cl_c1_codes_rows(int N, int B, int H, int W);
int avd_cl_c1_codes_cols(void);
int avd_cl_c1_apply_codes(const void* x, const void* wk, const float* bias, const float* scale,
                          const float* shift, void* z, unsigned* codes, int N, int B, int H, int W,
                          void* stream);
int avd_cl_c1_moments_codes(const void* x, const void* gz, const unsigned* codes, float* out,
                            int N, int B, int H, int W, void* stream);
int avd_cl_c1_codes_combine(const float* moments, const void* wk, const float* bias,
                            const float* gamma, const float* mean, const float* invstd,
                            long long count, float* dw, float* dgamma, float* dbeta, float* dbias,
                            float* coef, int G, void* stream);

/* ---- the same routed backward for the IMAGE conv1 (c1r5.hip; CentralUnimodalImage
 * conv1 -> bn1 -> relu -> maxpool, unimodal.py:127-141, 5x5 1->32 on 28x28, bf16).
 * avd_cl_c1r5_apply_codes: the pooled map z of avd_cl_c1_recompute pass 1 (bit-identical; a
 * pixel-major MFMA puts each pooling window in one lane) plus codes [N][14][14][8] u16:
 * word q of a window holds channels 4q..4q+3, nibble i (bits 4i..4i+3) = 1 + the window position
 * ((0,0),(0,1),(1,0),(1,1)) of the first argmax of relu(bn(y)) when that max is > 0, else 0.
 * avd_cl_c1r5_moments_codes: ONE pass over x, gz [N][14][14][32] and the codes -> per (row r,
 * group g) of avd_cl_c1r5_codes_rows rows, avd_cl_c1r5_codes_cols() floats: M[32][25] |
 * Gram[25][25] | S[25] | sum dz[32] at out[(r * G + g) * cols + ...] (reduce with avd_sum_rows);
 * the taps come from shifted copies of the image (no im2col gather).
 * avd_cl_c1r5_codes_combine: as avd_cl_c1_codes_combine for the 32 channels (G <= 32; the rows
 * functions return 0 beyond, and the engine then runs the recomputing moments pass). */
/* avd_cl_c1r5_stats: BN partial sums (sum y, sum y^2 of the bf16 y) of the recomputed image conv1
 * output as parts [32][G][R][2], R = avd_cl_c1r5_stats_rows (avd_bn_finalize's layout); the
 * pixel-major MFMA of avd_cl_c1r5_apply_codes, whose codes argument may be NULL (no backward). */
int avd_cl_c1r5_stats_rows(int N, int B, int H, int W);
int avd_cl_c1r5_stats(const void* x, const void* wk, const float* bias, float* out, int N, int B,
                      int H, int W, void* stream);
int avd_cl_c1r5_codes_rows(int N, int B, int H, int W);
int avd_cl_c1r5_codes_cols(void);
int avd_cl_c1r5_apply_codes(const void* x, const void* wk, const float* bias, const float* scale,
                            const float* shift, void* z, unsigned short* codes, int N, int B, int H,
                            int W, void* stream);
int avd_cl_c1r5_moments_codes(const void* x, const void* gz, const unsigned short* codes, float* out,
                              int N, int B, int H, int W, void* stream);
int avd_cl_c1r5_codes_combine(const float* moments, const void* wk, const float* bias,
                              const float* gamma, const float* mean, const float* invstd,
                              long long count, float* dw, float* dgamma, float* dbeta, float* dbias,
                              float* coef, int G, void* stream);

/* Timeline mark: marks[idx] = the device real-time counter (100 MHz ticks) when the stream
 * reaches this launch (tools: phase timing of a replayed step without a profiler). */
int avd_mark(unsigned long long* marks, int idx, void* stream);
/* Launch span marks around one launch site (bench.py's in-graph kernel duration): end = 0
 * stores the counter in spans[3 slot]; end = 1 adds (counter - spans[3 slot]) to spans[3 slot + 1]
 * and 1 to spans[3 slot + 2]. */
int avd_mark_span(unsigned long long* spans, int slot, int end, void* stream);
int avd_counters_add(long long* arena, const long long* idx, const long long* val, int n,
                     void* stream);

int avd_step_begin(long long* t, float* hyp, unsigned long long* seed_off, double b1, double b2,
                   unsigned long long seed_stride, void* stream);
int avd_adam_dev(float* p, const float* g, float* m, float* v, long long n, const float* hyp,
                 float b1, float b2, float eps, float wd, void* stream);
int avd_adamw_dev(float* p, const float* g, float* m, float* v, long long n, const float* hyp,
                  float b1, float b2, float eps, float wd, void* stream);

/* Eval-mode BatchNorm coefficients from running statistics: scale = gamma / sqrt(rv + eps),
 * shift = beta - rm * scale, [C] each (feed avd_cl_bn_relu_pool with G = 1). */
int avd_bn_eval_coef(const float* gamma, const float* beta, const float* running_mean,
                     const float* running_var, float eps, int C, float* scale, float* shift,
                     void* stream);

/* y += a*x over n floats (16-byte aligned): folds a scattered gradient slab into the local one
 * (global-negative contrastive losses, avdino/contrastive.py). */
int avd_axpy(float* y, const float* x, long long n, float a, void* stream);

/* out = sum(in[0..n)) in fixed order (loss reduction); out is one float. */
int avd_sum(const float* in, int n, float scale, float* out, void* stream);

/* ------------------------------------------------------------------ downstream evaluation
 * (training_structures/dino_train.py:47-102, 349-369) */

/* out[j] = sum_k x[j*D + k]^2 (the train-side term of the kNN distance). */
int avd_row_sqnorm(const float* x, int N, int D, float* out, void* stream);

/* kNN selection and vote (train_knn_classifier, dino_train.py:349-369: sklearn
 * KNeighborsClassifier(n_neighbors=K), brute-force euclidean, uniform weights).  For test row
 * i the distance to train row j ranks as xnorm[j] + S[i*ldS + j] where S = -2 Q X^T comes
 * from avd_gemm (the test row's own norm is common to the row).  With Q [M, D] / X [N, D]
 * (may be NULL) the min(16, N) best candidates of that ranking are re-ranked by their direct
 * distance sum_k (q_k - x_jk)^2 (no norm cancellation).  nbr [M, K] (may be NULL) receives the
 * K nearest train indices in increasing distance (ties: smaller index); pred [M] the class
 * with the most votes among labels[nbr] (ties: the smallest class, as sklearn's argmax over
 * class counts).  K <= 16, C <= 64; labels are class indices 0..C-1. */
int avd_knn_select(const float* S, long long ldS, const float* xnorm, int M, int N, int K,
                   const float* Q, const float* X, int D, const int64_t* labels, int C,
                   int64_t* nbr, int64_t* pred, void* stream);

/* idx[r] = argmax_j logits[r*ld + j], first maximum (torch.max(outputs, 1) in
 * compute_classification_metrics, dino_train.py:76). */
int avd_argmax_rows(const float* logits, long long ld, int R, int C, int64_t* idx, void* stream);

/* ------------------------------------------------------------------ audio conv1 from its patch Gram
 * The audio conv1 (CentralUnimodalAudio conv1: Conv2d(1, 8, 5, padding=2) on 112x112, bf16) has
 * Cin = 1, so y = w . x25 + b and its BatchNorm statistics follow exactly from the
 * weight-independent patch sums S = sum x25 and Gram = sum x25 x25^T per BN group:
 *   sum y = w . S + n b,   sum y^2 = w^T Gram w + 2 b w . S + n b^2.
 * avd_cl_c1_gram forms [avd_cl_c1_codes_rows][G][avd_cl_c1_gram_cols] partials (Gram 25x25 | S
 * 25; sum them with avd_sum_rows) in one MFMA pass over x -- no y, no per-element statistics;
 * avd_cl_c1_gram_finalize turns the row sums into avd_bn_finalize's outputs in float64 (mean,
 * invstd, BN scale / shift, running statistics in group order).  The routed backward then needs
 * no Gram of its own: avd_cl_c1_moments_codes_ng forms M and sum dz only (MOMC layout, Gram / S
 * slots zero) and avd_cl_c1_codes_combine_gram reads the forward's Gram. */
int avd_cl_c1_gram_cols(void);
int avd_cl_c1_gram(const void* x, float* out, int N, int B, int H, int W, void* stream);
int avd_cl_c1_gram_finalize(const float* gram, const void* wk, const float* bias, const float* gamma,
                            const float* beta, long long count, float eps, float momentum,
                            float* mean, float* invstd, float* scale, float* shift,
                            float* running_mean, float* running_var, int G, void* stream);
int avd_cl_c1_moments_codes_ng(const void* x, const void* gz, const unsigned* codes, float* out,
                               int N, int B, int H, int W, void* stream);
int avd_cl_c1_codes_combine_gram(const float* moments, const float* gram, const void* wk,
                                 const float* bias, const float* gamma, const float* mean,
                                 const float* invstd, long long count, float* dw, float* dgamma,
                                 float* dbeta, float* dbias, float* coef, int G, void* stream);

/* ------------------------------------------------------------------ routed 3x3 first layer
 * (28^2 and 112^2 run on the pixel-major / window-ordered kernels of c1s3.hip;
 * other shapes on c1w3.hip's recompute passes -- same contracts.)
 * The SimCLR / unimodal encoders' conv1 (audio_encoder / image_encoder, dino.py:18-73:
 * Conv2d(1, 32, 3, padding=1) -> BN2d -> ReLU -> MaxPool2d on 112x112 / 28x28, bf16) without a
 * stored conv output, backward routed by the forward's codes (the 3x3 counterpart of the
 * avd_cl_c1r5_* entry points): the BN -> ReLU -> pool pass also writes, per pooling window and
 * channel, the nibble 1 + (first argmax of relu(bn(y)) when > 0, else 0) -- u16 codes
 * [N][H/2][W/2][8]; the backward pass forms M = sum dz x9 (+ sum dz), Gram = sum x9 x9^T and
 * S = sum x9 per BN group from x, the pooled gradient and the codes (no y, no BN
 * coefficients), [avd_cl_c1r3_codes_rows][G][avd_cl_c1r3_codes_cols] partials (sum_rows), and
 * the float64 combine gives dW, dgamma, dbeta, dbias and the BN-backward coefficients. */
int avd_cl_c1r3_codes_rows(int N, int B, int H, int W, int Cout);
int avd_cl_c1r3_codes_cols(int Cout);
int avd_cl_c1r3_apply_codes(const void* x, const void* wk, const float* bias, const float* scale,
                            const float* shift, void* z, unsigned short* codes, int N, int B, int H,
                            int W, int Cout, void* stream);
int avd_cl_c1r3_moments_codes(const void* x, const void* wk, const void* gz, const unsigned short* codes,
                              float* out, int N, int B, int H, int W, int Cout, void* stream);
int avd_cl_c1r3_codes_combine(const float* moments, const void* wk, const float* bias,
                              const float* gamma, const float* mean, const float* invstd,
                              long long count, float* dw, float* dgamma, float* dbeta, float* dbias,
                              float* coef, int G, int Cout, void* stream);

/* ------------------------------------------------------------------ MX (block-scaled) fp8 convs
 * BASELINE config 5 ("fp8 MFMA conv path"): the mid-layer conv forward, input gradient AND
 * weight gradient of CentralUnimodalImage/Audio (unimodal.py:127-221; the F.conv2d and its
 * autograd dX / dW under the
 * reference's '16-mixed' precision, run_dino.py:360) on the block-scaled
 * v_mfma_scale_f32_16x16x128_f8f6f4 (gfx950, 2x the bf16 MFMA rate): OCP e4m3 operands with
 * E8M0 scales -- the weights one per (row, 32-k block), quantised per step by
 * avd_mx_weight_layout; the bf16 NHWC input quantised while staged with one power-of-two scale
 * per staged strip (its max maps into [128, 256): no saturation).  f32 accumulation; y / dX
 * bf16 NHWC; the forward's BatchNorm partial rows as avd_cl_conv_fwd's
 * ([Cout][N/B][avd_mx_stat_rows][2], optional pivot as avd_cl_conv_fwd_pv). */

/* Bytes of the e4m3 weight rows (rows of 16/64, k padded to 128) and of their E8M0 scales. */
long long avd_mx_weight_bytes(int Cout, int Cin, int K, int dgrad);
long long avd_mx_scale_bytes(int Cout, int Cin, int K, int dgrad);
/* W f32 [Cout][Cin][K][K] -> e4m3 rows + block scales; dgrad = 1: the input-gradient layout
 * (rows = input channels, taps flipped), as avd_cl_weight_layout. */
int avd_mx_weight_layout(const float* w, void* wq, void* wsc, int Cout, int Cin, int K, int dgrad,
                         void* stream);
/* n <= 16 layouts in one launch (a conv stack's per-step MX weights). */
int avd_mx_weight_layout_batch(int n, const float* const* w, void* const* wq, void* const* wsc,
                               const int* cout, const int* cin, const int* k, const int* dgrad,
                               void* stream);
/* 1 if the forward (dgrad 0) / input gradient (dgrad 1) of conv Cin -> Cout over H x W has an
 * MX kernel. */
int avd_mx_conv_serves(int Cin, int H, int W, int Cout, int K, int pad, int dgrad);
/* Samples per staged strip of that kernel (0: not served): it needs N % NS == 0, and a forward
 * writing BN partials B % NS == 0 (callers fall back to the bf16 kernels otherwise, e.g. the
 * last partial batch of the reference's DataLoader, get_data.py:464-467). */
int avd_mx_conv_ns(int Cin, int H, int W, int Cout, int K, int pad, int dgrad);
/* BN partial rows per group written by avd_mx_conv_fwd (0: not served). */
int avd_mx_stat_rows(int H, int W, int B, int K, int Cin, int Cout, int pad);
int avd_mx_conv_fwd(const void* x, const void* wq, const void* wsc, const float* bias,
                    const float* pivot, void* y, float* stats, int N, int B, int Cin, int H, int W,
                    int Cout, int K, int pad, void* stream);
/* dX [N][H][W][Cin] bf16 from dY [N][Ho][Wo][Cout] bf16 and the dgrad-layout MX weights. */
int avd_mx_conv_dgrad(const void* dy, const void* wq_d, const void* wsc_d, void* dx, int N, int Cin,
                      int H, int W, int Cout, int K, int pad, void* stream);
/* The conv's weight gradient (the autograd dW of nn.Conv2d) on the MX MFMA: x and dY bf16 NHWC
 * quantised while staged (one power-of-two scale per staged strip and operand), K = output
 * pixels; per-slab partials parts [avd_mx_wgrad_chunks][Cout][Cin][K][K] (sum: avd_sum_rows). */
int avd_mx_wgrad_chunks(int N, int Cin, int H, int Cout, int K, int pad);
int avd_mx_conv_wgrad(const void* x, const void* dy, float* parts, int N, int Cin, int H, int W,
                      int Cout, int K, int pad, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* AVDINO_H */
