// C ABI of the channels-last (NHWC) conv-block path (include/avdino.h, "avd_cl_*").
#include <cstdlib>

#include "common.h"

int avd_cl_layout_rows_impl(int O);
int avd_cl_stat_rows_impl(int Ho, int Wo, int B, int K, int Cin, int Cout, int dt);
int avd_cl_weight_layout_impl(const float* w, void* wk, int dt, int Cout, int Cin, int K,
                              int dgrad, hipStream_t st);
int avd_cl_weight_layout_batch_impl(int n, const float* const* w, void* const* wk,
                                    const int* cout, const int* cin, const int* k,
                                    const int* dgrad, int dt, hipStream_t st);
int avd_cl_conv_fwd_impl(const void* x, const void* wk, const float* bias, void* y, float* stats,
                         int dt, int N, int B, int Cin, int H, int W, int Cout, int K, int pad,
                         hipStream_t st, const float* pivot);
int avd_ws_stat_rows(int Ho, int Wo, int B, int K, int Cin, int Cout, int dt);
int avd_cl_conv_dgrad_impl(const void* dy, const void* wk_d, void* dx, int dt, int N, int Cin,
                           int H, int W, int Cout, int K, int pad, hipStream_t st);
int avd_cl_wgrad_chunks_impl(int N, int Cout, int Cin, int K);
int avd_cl_conv_wgrad_impl(const void* x, const void* dy, int dt, float* parts, int N, int Cin,
                           int H, int W, int Cout, int K, int pad, hipStream_t st);
int avd_cl_bn_relu_pool_impl(const void* y, int dt, const float* scale, const float* shift,
                             void* out, int mode, int N, int B, int C, int H, int W,
                             hipStream_t st);
int avd_cl_bn_bwd_rows_impl(int B, int C, int H, int W, int dt);
int avd_cl_bn_bwd_reduce_impl(const void* y, int dt, const void* gout, int mode,
                              const float* scale, const float* shift, const float* mean,
                              const float* invstd, float* parts, int N, int B, int C, int H,
                              int W, hipStream_t st);
int avd_cl_bn_bwd_apply_impl(const void* y, int dt, const void* gout, int mode,
                             const float* scale, const float* shift, const float* coef, void* dy,
                             int N, int B, int C, int H, int W, hipStream_t st);

bool avd_c1p8_eligible(int dt, int Cin, int Cout, int K, int Ho, int Wo);
int avd_c1p8_wgrad_slabs(int N, int H);
int avd_c1p8_bwd_apply_wgrad(const void* y, const void* gout, const float* scale,
                             const float* shift, const float* coef, const void* x, float* parts,
                             int N, int B, int H, int W, hipStream_t st);

int avd_c1_codes_rows(int N, int B);
int avd_c1_codes_cols();
int avd_c1_apply_codes_launch(const void* x, const void* wk, const float* bias, const float* scale,
                              const float* shift, void* z, unsigned* codes, int N, int B, int H,
                              int W, hipStream_t st);
int avd_c1_moments_codes_launch(const void* x, const void* gz, const unsigned* codes, float* out,
                                int N, int B, int H, int W, hipStream_t st);
int avd_c1_codes_combine_launch(const float* m, const void* wk, const float* bias,
                                const float* gamma, const float* mean, const float* invstd,
                                long long count, float* dw, float* dgamma, float* dbeta,
                                float* dbias, float* coef, int G, hipStream_t st,
                                const float* gram = nullptr);
int avd_c1_gram_launch(const void* x, float* out, int N, int B, int H, int W, hipStream_t st);
int avd_c1_moments_nogram_launch(const void* x, const void* gz, const unsigned* codes, float* out,
                                 int N, int B, int H, int W, hipStream_t st);
int avd_c1_gram_cols();
int avd_c1_gram_finalize_launch(const float* gram, const void* wk, const float* bias,
                                const float* gamma, const float* beta, float eps, float momentum,
                                long long count, float* mean, float* invstd, float* scale,
                                float* shift, float* rm, float* rv, int G, hipStream_t st);

int avd_c1r_rows(int pass, int N, int B, int H);
int avd_c1p8_moment_cols();
int avd_c1p8_combine(const float* m, const float* coef, const void* wk, const float* bias,
                     float* dw, int G, hipStream_t st);
int avd_c1r_launch(int pass, const void* x, const void* wk, const float* bias, const float* scale,
                   const float* shift, const float* mean, const float* invstd, const float* coef,
                   const void* gz, void* z, float* out, int N, int B, int H, int W,
                   hipStream_t st);

namespace {
bool dt_ok(int dt) { return dt == AVD_F32 || dt == AVD_BF16; }
}  // namespace


int avd_cl_bn_bwd_reduce_pooled_impl(const void* y, int dt, const void* pooled, const void* gout,
                                     int mode, const float* gamma, const float* beta,
                                     const float* mean, const float* invstd, float* parts, int N,
                                     int B, int C, int H, int W, hipStream_t st);


extern "C" {

int avd_cl_weight_elems(int Cout, int Cin, int K, int dgrad) {
  const int O = dgrad ? Cin : Cout, C = dgrad ? Cout : Cin;
  return avd_cl_layout_rows_impl(O) * avd_cdiv(K * K * C, 32) * 32;
}

int avd_cl_weight_layout(const float* w, void* wk, int dt, int Cout, int Cin, int K, int dgrad,
                         void* stream) {
  if (!w || !wk || !dt_ok(dt)) return AVD_ERR_ARG;
  if (Cout <= 0 || Cin <= 0 || K <= 0) return AVD_ERR_SHAPE;
  return avd_cl_weight_layout_impl(w, wk, dt, Cout, Cin, K, dgrad, avd_stream(stream));
}

int avd_cl_weight_layout_batch(int n, const float* const* w, void* const* wk, const int* cout,
                               const int* cin, const int* k, const int* dgrad, int dt,
                               void* stream) {
  if (!w || !wk || !cout || !cin || !k || !dgrad || !dt_ok(dt)) return AVD_ERR_ARG;
  for (int e = 0; e < n; ++e)
    if (cout[e] <= 0 || cin[e] <= 0 || k[e] <= 0) return AVD_ERR_SHAPE;
  return avd_cl_weight_layout_batch_impl(n, w, wk, cout, cin, k, dgrad, dt, avd_stream(stream));
}

int avd_c1w3_slabs(int dt, int N, int Cin, int H, int W, int Cout, int K, int pad);
int avd_c1w3_apply_wgrad(const void* y, const void* gout, const float* scale, const float* shift,
                         const float* coef, const void* x, float* parts, int N, int B, int H,
                         int W, int Cout, hipStream_t st);

int avd_cl_apply_wgrad_slabs(int dt, int N, int Cin, int H, int W, int Cout, int K, int pad) {
  // the first 3x3 layer of the SimCLR / unimodal encoders (c1w3.hip)
  if (const int s = avd_c1w3_slabs(dt, N, Cin, H, W, Cout, K, pad)) return s;
  if (!avd_c1p8_eligible(dt, Cin, Cout, K, H, W) || pad != 2 || W > 112) return 0;
  return avd_c1p8_wgrad_slabs(N, H);
}

int avd_cl_bn_bwd_apply_wgrad(const void* y, const void* gout, const float* scale,
                              const float* shift, const float* coef, const void* x, float* parts,
                              int dt, int N, int B, int Cin, int H, int W, int Cout, int K, int pad,
                              void* stream) {
  if (!y || !gout || !scale || !shift || !coef || !x || !parts) return AVD_ERR_ARG;
  if (N <= 0 || B <= 0 || N % B) return AVD_ERR_SHAPE;
  if (avd_cl_apply_wgrad_slabs(dt, N, Cin, H, W, Cout, K, pad) == 0) return AVD_ERR_SHAPE;
  if (avd_c1w3_slabs(dt, N, Cin, H, W, Cout, K, pad))
    return avd_c1w3_apply_wgrad(y, gout, scale, shift, coef, x, parts, N, B, H, W, Cout,
                                avd_stream(stream));
  return avd_c1p8_bwd_apply_wgrad(y, gout, scale, shift, coef, x, parts, N, B, H, W,
                                  avd_stream(stream));
}

int avd_c1r3_rows(int pass, int dt, int N, int B, int Cin, int H, int W, int Cout, int K, int pad);
int avd_c1r3_launch(int pass, const void* x, const void* wk, const float* bias, const float* scale,
                    const float* shift, const float* mean, const float* invstd, const float* coef,
                    const void* gz, void* z, float* out, int N, int B, int H, int W, int Cout, int K,
                    hipStream_t st, unsigned short* codes = nullptr);

int avd_c1r3_combine(const float* m, const float* coef, const void* wk, const float* bias,
                     float* dw, int G, int Cout, int K, hipStream_t st);

int avd_cl_c1_recompute_rows(int pass, int dt, int N, int B, int Cin, int H, int W, int Cout,
                             int K, int pad) {
  if (pass < 0 || pass > 4 || B <= 0 || N % B) return 0;
  // the 3x3 encoders' first layer (c1w3.hip); pass 4 (reduce + weight-gradient moments) only there
  if (const int r = avd_c1r3_rows(pass, dt, N, B, Cin, H, W, Cout, K, pad)) return r;
  if (!avd_c1p8_eligible(dt, Cin, Cout, K, H, W) || pad != 2 || W > 112) return 0;
  return avd_c1r_rows(pass, N, B, H);
}

int avd_cl_c1_recompute(int pass, const void* x, const void* wk, const float* bias,
                        const float* scale, const float* shift, const float* mean,
                        const float* invstd, const float* coef, const void* gz, void* z,
                        float* out, int dt, int N, int B, int Cin, int H, int W, int Cout, int K,
                        int pad, void* stream) {
  if (!x || !wk) return AVD_ERR_ARG;
  if (avd_cl_c1_recompute_rows(pass, dt, N, B, Cin, H, W, Cout, K, pad) == 0) return AVD_ERR_SHAPE;
  const bool need_bn = pass != 0, need_g = pass >= 2;
  if ((need_bn && (!scale || !shift)) || (pass == 1 && !z) || (pass != 1 && !out) ||
      (need_g && !gz) || ((pass == 2 || pass == 4) && (!mean || !invstd)) || (pass == 3 && !coef))
    return AVD_ERR_ARG;
  if (avd_c1r3_rows(pass, dt, N, B, Cin, H, W, Cout, K, pad))
    return avd_c1r3_launch(pass, x, wk, bias, scale, shift, mean, invstd, coef, gz, z, out, N, B,
                           H, W, Cout, K, avd_stream(stream));
  return avd_c1r_launch(pass, x, wk, bias, scale, shift, mean, invstd, coef, gz, z, out, N, B, H,
                        W, avd_stream(stream));
}

int avd_cl_c1_recompute_combine(const float* moments, const float* coef, const void* wk,
                                const float* bias, float* dw, int G, int Cout, int K, void* stream) {
  if (!moments || !coef || !wk || !dw) return AVD_ERR_ARG;
  if (G <= 0 || (Cout != 8 && Cout != 16 && Cout != 32 && Cout != 64) || (K != 3 && K != 5))
    return AVD_ERR_SHAPE;
  if (Cout == 8)   // the 5x5 audio conv1 (conv_c1p.hip)
    return K == 5 ? avd_c1p8_combine(moments, coef, wk, bias, dw, G, avd_stream(stream)) : AVD_ERR_SHAPE;
  return avd_c1r3_combine(moments, coef, wk, bias, dw, G, Cout, K, avd_stream(stream));
}

namespace {
bool c1_codes_shape(int N, int B, int H, int W) {
  return N > 0 && B > 0 && N % B == 0 && N / B <= 32 && avd_c1p8_eligible(AVD_BF16, 1, 8, 5, H, W) &&
         W <= 112 && H % 2 == 0 && W % 2 == 0;   // <= 32 BN groups: the combine's table
}
}  // namespace

int avd_cl_c1_codes_rows(int N, int B, int H, int W) {
  return c1_codes_shape(N, B, H, W) ? avd_c1_codes_rows(N, B) : 0;
}

int avd_cl_c1_codes_cols(void) { return avd_c1_codes_cols(); }

int avd_cl_c1_apply_codes(const void* x, const void* wk, const float* bias, const float* scale,
                          const float* shift, void* z, unsigned* codes, int N, int B, int H, int W,
                          void* stream) {
  if (!x || !wk || !scale || !shift || !z || !codes) return AVD_ERR_ARG;
  if (!c1_codes_shape(N, B, H, W)) return AVD_ERR_SHAPE;
  return avd_c1_apply_codes_launch(x, wk, bias, scale, shift, z, codes, N, B, H, W,
                                   avd_stream(stream));
}

int avd_cl_c1_moments_codes(const void* x, const void* gz, const unsigned* codes, float* out,
                            int N, int B, int H, int W, void* stream) {
  if (!x || !gz || !codes || !out) return AVD_ERR_ARG;
  if (!c1_codes_shape(N, B, H, W)) return AVD_ERR_SHAPE;
  return avd_c1_moments_codes_launch(x, gz, codes, out, N, B, H, W, avd_stream(stream));
}

int avd_cl_c1_codes_combine(const float* moments, const void* wk, const float* bias,
                            const float* gamma, const float* mean, const float* invstd,
                            long long count, float* dw, float* dgamma, float* dbeta, float* dbias,
                            float* coef, int G, void* stream) {
  if (!moments || !wk || !gamma || !mean || !invstd || !dw) return AVD_ERR_ARG;
  if (G <= 0 || count <= 1) return AVD_ERR_SHAPE;
  return avd_c1_codes_combine_launch(moments, wk, bias, gamma, mean, invstd, count, dw, dgamma,
                                     dbeta, dbias, coef, G, avd_stream(stream));
}

// the audio conv1's statistics from its patch Gram matrix (include/avdino.h)
int avd_cl_c1_gram_cols(void) { return avd_c1_gram_cols(); }

int avd_cl_c1_gram(const void* x, float* out, int N, int B, int H, int W, void* stream) {
  if (!x || !out) return AVD_ERR_ARG;
  if (!c1_codes_shape(N, B, H, W)) return AVD_ERR_SHAPE;
  return avd_c1_gram_launch(x, out, N, B, H, W, avd_stream(stream));
}

int avd_cl_c1_gram_finalize(const float* gram, const void* wk, const float* bias, const float* gamma,
                            const float* beta, long long count, float eps, float momentum,
                            float* mean, float* invstd, float* scale, float* shift,
                            float* running_mean, float* running_var, int G, void* stream) {
  if (!gram || !wk || !gamma || !beta || !mean || !invstd || !scale || !shift) return AVD_ERR_ARG;
  if (G <= 0 || count <= 1) return AVD_ERR_SHAPE;
  return avd_c1_gram_finalize_launch(gram, wk, bias, gamma, beta, eps, momentum, count, mean, invstd,
                                     scale, shift, running_mean, running_var, G, avd_stream(stream));
}

int avd_cl_c1_moments_codes_ng(const void* x, const void* gz, const unsigned* codes, float* out,
                               int N, int B, int H, int W, void* stream) {
  if (!x || !gz || !codes || !out) return AVD_ERR_ARG;
  if (!c1_codes_shape(N, B, H, W)) return AVD_ERR_SHAPE;
  return avd_c1_moments_nogram_launch(x, gz, codes, out, N, B, H, W, avd_stream(stream));
}

int avd_cl_c1_codes_combine_gram(const float* moments, const float* gram, const void* wk,
                                 const float* bias, const float* gamma, const float* mean,
                                 const float* invstd, long long count, float* dw, float* dgamma,
                                 float* dbeta, float* dbias, float* coef, int G, void* stream) {
  if (!moments || !gram || !wk || !gamma || !mean || !invstd || !dw) return AVD_ERR_ARG;
  if (G <= 0 || count <= 1) return AVD_ERR_SHAPE;
  return avd_c1_codes_combine_launch(moments, wk, bias, gamma, mean, invstd, count, dw, dgamma,
                                     dbeta, dbias, coef, G, avd_stream(stream), gram);
}

int avd_cl_c1_moment_cols(int Cout, int K) {
  if (Cout == 8) return K == 5 ? avd_c1p8_moment_cols() : 0;
  if ((Cout == 16 || Cout == 32 || Cout == 64) && (K == 3 || K == 5)) return Cout * K * K + K * K * (K * K + 1);
  return 0;
}

int avd_cl_stat_rows(int Ho, int Wo, int B, int K, int Cin, int Cout, int dt) {
  return avd_cl_stat_rows_impl(Ho, Wo, B, K, Cin, Cout, dt);
}

int avd_cl_conv_fwd(const void* x, const void* wk, const float* bias, void* y, float* stats,
                    int dt, int N, int B, int Cin, int H, int W, int Cout, int K, int pad,
                    void* stream) {
  return avd_cl_conv_fwd_pv(x, wk, bias, nullptr, y, stats, dt, N, B, Cin, H, W, Cout, K, pad,
                            stream);
}

int avd_cl_stat_pivot(int Ho, int Wo, int B, int K, int Cin, int Cout, int dt) {
  return avd_ws_stat_rows(Ho, Wo, B, K, Cin, Cout, dt) > 0;
}

int avd_cl_conv_fwd_pv(const void* x, const void* wk, const float* bias, const float* pivot,
                       void* y, float* stats, int dt, int N, int B, int Cin, int H, int W, int Cout,
                       int K, int pad, void* stream) {
  if (!x || !wk || !y || !dt_ok(dt)) return AVD_ERR_ARG;
  if (N <= 0 || B <= 0 || (K != 3 && K != 5)) return AVD_ERR_SHAPE;
  return avd_cl_conv_fwd_impl(x, wk, bias, y, stats, dt, N, B, Cin, H, W, Cout, K, pad,
                              avd_stream(stream), stats ? pivot : nullptr);
}

int avd_cl_conv_dgrad(const void* dy, const void* wk_d, void* dx, int dt, int N, int Cin, int H,
                      int W, int Cout, int K, int pad, void* stream) {
  if (!dy || !wk_d || !dx || !dt_ok(dt)) return AVD_ERR_ARG;
  if (N <= 0 || (K != 3 && K != 5)) return AVD_ERR_SHAPE;
  return avd_cl_conv_dgrad_impl(dy, wk_d, dx, dt, N, Cin, H, W, Cout, K, pad, avd_stream(stream));
}

int avd_cl_bn_bwd_reduce_pooled(const void* y, int dt, const void* pooled, const void* gout,
                                int mode, const float* gamma, const float* beta, const float* mean,
                                const float* invstd, float* parts, int N, int B, int C, int H,
                                int W, void* stream) {
  if (!y || !pooled || !gout || !gamma || !beta || !mean || !invstd || !parts || !dt_ok(dt))
    return AVD_ERR_ARG;
  if (N <= 0 || B <= 0 || H < 2 || W < 2) return AVD_ERR_SHAPE;
  return avd_cl_bn_bwd_reduce_pooled_impl(y, dt, pooled, gout, mode, gamma, beta, mean, invstd,
                                          parts, N, B, C, H, W, avd_stream(stream));
}

int avd_cl_wgrad_chunks(int N, int Cout, int Cin, int K) {
  return avd_cl_wgrad_chunks_impl(N, Cout, Cin, K);
}

int avd_cl_conv_wgrad(const void* x, const void* dy, int dt, float* dw_parts, int N, int Cin,
                      int H, int W, int Cout, int K, int pad, void* stream) {
  if (!x || !dy || !dw_parts || !dt_ok(dt)) return AVD_ERR_ARG;
  if (N <= 0 || (K != 3 && K != 5)) return AVD_ERR_SHAPE;
  return avd_cl_conv_wgrad_impl(x, dy, dt, dw_parts, N, Cin, H, W, Cout, K, pad,
                                avd_stream(stream));
}

int avd_cl_bn_relu_pool(const void* y, int dt, const float* scale, const float* shift, void* out,
                        int mode, int N, int B, int C, int H, int W, void* stream) {
  if (!y || !scale || !shift || !out || !dt_ok(dt)) return AVD_ERR_ARG;
  if (N <= 0 || B <= 0) return AVD_ERR_SHAPE;
  return avd_cl_bn_relu_pool_impl(y, dt, scale, shift, out, mode, N, B, C, H, W,
                                  avd_stream(stream));
}

int avd_cl_bn_bwd_rows(int B, int C, int H, int W, int dt) {
  return avd_cl_bn_bwd_rows_impl(B, C, H, W, dt);
}

int avd_cl_bn_bwd_reduce(const void* y, int dt, const void* gout, int mode, const float* scale,
                         const float* shift, const float* mean, const float* invstd, float* parts,
                         int N, int B, int C, int H, int W, void* stream) {
  if (!y || !gout || !scale || !shift || !mean || !invstd || !parts || !dt_ok(dt))
    return AVD_ERR_ARG;
  if (N <= 0 || B <= 0) return AVD_ERR_SHAPE;
  return avd_cl_bn_bwd_reduce_impl(y, dt, gout, mode, scale, shift, mean, invstd, parts, N, B, C,
                                   H, W, avd_stream(stream));
}

int avd_cl_bn_bwd_apply(const void* y, int dt, const void* gout, int mode, const float* scale,
                        const float* shift, const float* coef, void* dy, int N, int B, int C,
                        int H, int W, void* stream) {
  if (!y || !gout || !scale || !shift || !coef || !dy || !dt_ok(dt)) return AVD_ERR_ARG;
  if (N <= 0 || B <= 0) return AVD_ERR_SHAPE;
  return avd_cl_bn_bwd_apply_impl(y, dt, gout, mode, scale, shift, coef, dy, N, B, C, H, W,
                                  avd_stream(stream));
}

}  // extern "C"
