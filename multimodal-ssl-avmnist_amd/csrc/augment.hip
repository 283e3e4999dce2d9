// Device-side view augmentation: the per-sample CPU transform chains of
// MultiModalAugmentation (AVMNIST_Experiments/utils/get_data.py:110-257) as one gather kernel.
//
// The host draws every random parameter (avdino/augment.py follows torchvision's / torchaudio's
// get_params rules) into one record per (sample, view); the device does the pixel work.  One
// block builds one output view: the sample's source row (H*W bytes) is gathered by its dataset
// index, normalised through the dataset's byte->f32 table and staged in LDS once, then every
// output pixel walks the chain backwards (output -> affine -> rotation -> masks -> time stretch
// -> crop -> source) with the reference's interpolation at each stage.  HBM traffic per view is
// H*W source bytes + 4*H*W output bytes; the kernel is write-bound.
//
// Floating-point contraction is off so the coordinate and interpolation arithmetic rounds the
// way the numpy restatement in oracle/augment.py does (bit-identical outside the noise term).
#include "common.h"

using namespace avd;

namespace {

constexpr int kThreads = 256;
constexpr int kMaxHW = 112 * 112;

__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  x ^= x >> 31;
  return x;
}

// Two standard normals for the pixel pair (2q, 2q+1) of a record: one Box-Muller draw over a
// 64-bit counter hash of (seed, record, q) -- the cosine for the even pixel, the sine for the odd
// one (independent N(0,1) values; one hash, one log, one sqrt per two pixels).
__device__ __forceinline__ float2 gauss2(unsigned long long seed, unsigned rec, unsigned q) {
#pragma clang fp contract(off)
  const unsigned long long r = mix64(seed ^ mix64(((unsigned long long)rec << 32) | q));
  const float u1 = (float)((r >> 40) + 1ull) * 5.9604644775390625e-8f;  // (0, 1]
  const float u2 = (float)((r >> 16) & 0xFFFFFFull) * 5.9604644775390625e-8f;
  const float mag = sqrtf(-2.0f * logf(u1)), ang = 6.2831855f * u2;
  return make_float2(mag * cosf(ang), mag * sinf(ang));
}

// Nearest-neighbour inverse map of a torchvision affine / rotation (grid_sample, zero padding,
// align_corners=False): src = M (p - c) + t + c, c = ((W-1)/2, (H-1)/2), rounded half-to-even.
__device__ __forceinline__ bool affine_nearest(const float* m, float cx, float cy, int W, int H,
                                               int& x, int& y) {
#pragma clang fp contract(off)
  const float dx = (float)x - cx, dy = (float)y - cy;
  const float sx = ((m[0] * dx + m[1] * dy) + m[2]) + cx;
  const float sy = ((m[3] * dx + m[4] * dy) + m[5]) + cy;
  const float rx = rintf(sx), ry = rintf(sy);
  if (!(rx >= 0.0f && rx <= (float)(W - 1) && ry >= 0.0f && ry <= (float)(H - 1))) return false;
  x = (int)rx;
  y = (int)ry;
  return true;
}

struct View {
  const float* img;   // LDS, [H, W] normalised source
  const uint8_t* gsrc;  // GLB kernels: the source row's bytes in global memory
  const float* glut;    //   and the byte -> f32 table
  int H, W;
  bool crop;
  int top, left, ch, cw;
  float sh, sw;       // ch / H, cw / W
};

// RandomResizedCrop output pixel (r, c): bilinear (align_corners=False, source index clamped
// at 0 and at the crop's last row/column) inside the integer crop box.
template <bool GLB = false>
__device__ __forceinline__ float src_px(const View& v, int i) {
  if constexpr (GLB) return v.glut[v.gsrc[i]];
  else return v.img[i];
}

template <bool GLB = false>
__device__ __forceinline__ float crop_sample(const View& v, int r, int c) {
#pragma clang fp contract(off)
  if (!v.crop) return src_px<GLB>(v, r * v.W + c);
  float sy = ((float)r + 0.5f) * v.sh - 0.5f;
  float sx = ((float)c + 0.5f) * v.sw - 0.5f;
  sy = sy < 0.0f ? 0.0f : sy;
  sx = sx < 0.0f ? 0.0f : sx;
  const int y0 = (int)sy, x0 = (int)sx;
  const int y1 = y0 + 1 < v.ch ? y0 + 1 : v.ch - 1;
  const int x1 = x0 + 1 < v.cw ? x0 + 1 : v.cw - 1;
  const float ly = sy - (float)y0, lx = sx - (float)x0;
  const float hy = 1.0f - ly, hx = 1.0f - lx;
  const int r0 = (v.top + y0) * v.W + v.left, r1 = (v.top + y1) * v.W + v.left;
  return hy * (hx * src_px<GLB>(v, r0 + x0) + lx * src_px<GLB>(v, r0 + x1)) +
         ly * (hx * src_px<GLB>(v, r1 + x0) + lx * src_px<GLB>(v, r1 + x1));
}

// CHK (avd_augment_views_lds_check, a diagnostic): after the pixel loop every thread re-derives
// its staged source floats and the byte table from global memory and counts the LDS words that no
// longer hold them into chk[0] (first bad word index in chk[1], the block in chk[2]).
template <typename TO, bool CHK = false, bool GLB = false>
__global__ __launch_bounds__(kThreads) void augment_kernel(
    const uint8_t* __restrict__ src, const int64_t* __restrict__ idx, int V, int B, int H, int W,
    const float* __restrict__ lut, const float* __restrict__ recs, const uint32_t* __restrict__ gm,
    int gm_words, int group, unsigned long long seed, int order, TO* __restrict__ out,
    int* __restrict__ chk = nullptr, float* __restrict__ seen = nullptr) {
#pragma clang fp contract(off)
  __shared__ float s_img[kMaxHW];
  __shared__ float s_lut[256];
  const int rid = blockIdx.x;  // record = b * V + v
  const int b = rid / V, v = rid - b * V;
  const int HW = H * W;
  const float* rec = recs + (size_t)rid * AVD_AUG_REC;

  const uint32_t* row = reinterpret_cast<const uint32_t*>(src + (size_t)idx[b] * HW);
  if constexpr (!GLB) {
    s_lut[threadIdx.x] = lut[threadIdx.x];
    __syncthreads();
    for (int i = threadIdx.x; i < HW / 4; i += kThreads) {
      const uint32_t w4 = row[i];
      s_img[4 * i + 0] = s_lut[w4 & 0xFF];
      s_img[4 * i + 1] = s_lut[(w4 >> 8) & 0xFF];
      s_img[4 * i + 2] = s_lut[(w4 >> 16) & 0xFF];
      s_img[4 * i + 3] = s_lut[w4 >> 24];
    }
    __syncthreads();
  }

  const int flags = (int)rec[AVD_AUG_FLAGS];
  View vw;
  vw.img = s_img;
  vw.gsrc = reinterpret_cast<const uint8_t*>(row);
  vw.glut = lut;
  vw.H = H;
  vw.W = W;
  vw.crop = flags & 1;
  vw.top = (int)rec[AVD_AUG_CROP + 0];
  vw.left = (int)rec[AVD_AUG_CROP + 1];
  vw.ch = (int)rec[AVD_AUG_CROP + 2];
  vw.cw = (int)rec[AVD_AUG_CROP + 3];
  vw.sh = (float)vw.ch / (float)H;
  vw.sw = (float)vw.cw / (float)W;
  const bool aff = flags & 2, rot = flags & 4, tw = flags & 8;
  float maff[6], mrot[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    maff[k] = rec[AVD_AUG_AFF + k];
    mrot[k] = rec[AVD_AUG_ROT + k];
  }
  const float rate = rec[AVD_AUG_RATE];
  const int f0 = (int)rec[AVD_AUG_FMASK], f1 = (int)rec[AVD_AUG_FMASK + 1];
  const int t0 = (int)rec[AVD_AUG_TMASK], t1 = (int)rec[AVD_AUG_TMASK + 1];
  const float nstd = rec[AVD_AUG_NOISE];
  const int gmrow = (int)rec[AVD_AUG_GM];
  const int et = (int)rec[AVD_AUG_ERASE], el = (int)rec[AVD_AUG_ERASE + 1];
  const int eh = (int)rec[AVD_AUG_ERASE + 2], ew = (int)rec[AVD_AUG_ERASE + 3];
  const float cx = (float)(W - 1) * 0.5f, cy = (float)(H - 1) * 0.5f;
  const uint32_t* gmr = (gm && gmrow >= 0) ? gm + (size_t)gmrow * gm_words : nullptr;
  const int gw = group > 0 ? W / group : 1;
  TO* o = out + (order == 0 ? (size_t)rid : (size_t)v * B + b) * HW;

  // a thread builds the pixel pair (2q, 2q+1): W is even, so a pair never straddles a row; it
  // shares the row index, one noise draw and one (2 x bf16 / 2 x f32) store
  const FastDiv divw(W / 2), divg(group > 0 ? group : 1);
  for (int q = threadIdx.x; q < HW / 2; q += kThreads) {
    const int y = divw.div(q), x0 = 2 * (q - y * (W / 2));
    float2 g2 = make_float2(0.f, 0.f);
    if (nstd != 0.0f) g2 = gauss2(seed, (unsigned)rid, (unsigned)q);
    const int gy = gmr ? divg.div(y) * gw : 0;
    float v2[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int x = x0 + e;
      int qx = x, qy = y;
      bool ok = true;
      if (aff) ok = affine_nearest(maff, cx, cy, W, H, qx, qy);
      if (ok && rot) ok = affine_nearest(mrot, cx, cy, W, H, qx, qy);
      float val = 0.0f;
      if (ok && !(qy >= f0 && qy < f1) && !(qx >= t0 && qx < t1)) {
        if (tw) {
          // |phase_vocoder(spec, rate)|[c] = a*|s[i0+1]| + (1-a)*|s[i0]|, t = c*rate, zero past
          // the input's end (torchaudio pads two zero frames); ceil(W/rate) output frames.
          const float t = (float)qx * rate;
          if (t < (float)W) {
            const int i0 = (int)t;
            const float a = t - (float)i0;
            const float s0 = fabsf(crop_sample<GLB>(vw, qy, i0));
            const float s1 = i0 + 1 < W ? fabsf(crop_sample<GLB>(vw, qy, i0 + 1)) : 0.0f;
            val = a * s1 + (1.0f - a) * s0;
          }
        } else {
          val = crop_sample<GLB>(vw, qy, qx);
        }
      }
      if (eh > 0 && y >= et && y < et + eh && x >= el && x < el + ew) val = 0.0f;
      if (nstd != 0.0f) val = val + (e ? g2.y : g2.x) * nstd;
      if (gmr) {
        const int g = gy + divg.div(x);
        if ((gmr[g >> 5] >> (g & 31)) & 1u) val = val * 0.0f;
      }
      v2[e] = val;
    }
    if constexpr (sizeof(TO) == 4)
      reinterpret_cast<float2*>(o)[q] = make_float2(v2[0], v2[1]);
    else      // bf16 straight into the engine's staged view-major input
      reinterpret_cast<uint32_t*>(o)[q] = pack_bf16x2(v2[0], v2[1]);
  }
  if constexpr (CHK && !GLB) {
    if (threadIdx.x == 0) {   // the record as this block used it
      float* sr = seen + (size_t)rid * AVD_AUG_REC;
      sr[AVD_AUG_FLAGS] = (float)flags;
      sr[AVD_AUG_CROP + 0] = (float)vw.top; sr[AVD_AUG_CROP + 1] = (float)vw.left;
      sr[AVD_AUG_CROP + 2] = (float)vw.ch; sr[AVD_AUG_CROP + 3] = (float)vw.cw;
      for (int k = 0; k < 6; ++k) { sr[AVD_AUG_AFF + k] = maff[k]; sr[AVD_AUG_ROT + k] = mrot[k]; }
      sr[AVD_AUG_RATE] = rate;
      sr[AVD_AUG_FMASK] = (float)f0; sr[AVD_AUG_FMASK + 1] = (float)f1;
      sr[AVD_AUG_TMASK] = (float)t0; sr[AVD_AUG_TMASK + 1] = (float)t1;
      sr[AVD_AUG_NOISE] = nstd;
      sr[AVD_AUG_GM] = (float)gmrow;
      sr[AVD_AUG_ERASE] = (float)et; sr[AVD_AUG_ERASE + 1] = (float)el;
      sr[AVD_AUG_ERASE + 2] = (float)eh; sr[AVD_AUG_ERASE + 3] = (float)ew;
    }
    __syncthreads();
    int nbad = 0, first = -1;
    if (__float_as_uint(s_lut[threadIdx.x]) != __float_as_uint(lut[threadIdx.x])) {
      ++nbad;
      first = kMaxHW + threadIdx.x;
    }
    for (int i = threadIdx.x; i < HW / 4; i += kThreads) {
      const uint32_t w4 = row[i];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (__float_as_uint(s_img[4 * i + j]) != __float_as_uint(lut[(w4 >> (8 * j)) & 0xFF])) {
          ++nbad;
          if (first < 0) first = 4 * i + j;
        }
    }
    if (nbad) {
      atomicAdd(chk, nbad);
      chk[1] = first;
      chk[2] = rid;
    }
  }
}

enum { SK_CROP = 0, SK_TWARP, SK_FMASK, SK_TMASK, SK_ROT, SK_AFF, SK_ERASE, SK_NOISE, SK_GMASK };
constexpr int kMaxStages = 9, kStageF = 8, kMaxGroups = 1024;

// ----------------------------------------------------------------------------- any stage order
// transforms.Compose applies a chain in its own order, and the reference's own config
// (configs/config_multimodal_dino.yaml best_augments -> MultiModalAugmentation(augment_values=...),
// get_data.py:195-231) orders its audio chains by YAML key: frequency mask, noise, time mask,
// time stretch, crop, affine -- not the fixed order the gather kernel above walks backwards.
// This kernel runs the chain forwards, one stage at a time, over the view held in LDS (f32):
// each applied stage reads the previous stage's whole image, exactly as each torchvision /
// torchaudio module reads its predecessor's output.  A thread owns pixels tid + k*256; the
// resampling stages (crop, time stretch, rotation, affine) gather into registers, then a
// barrier, then overwrite the image; the value stages (masks, erasing, noise, groups) update
// their own pixels in place.  Same per-pixel formulas as the gather kernel, so a chain in the
// fixed order gives bit-identical views either way.
struct Prog { int kind[kMaxStages]; int n; };

template <typename TO, int NPT>
__global__ __launch_bounds__(kThreads) void augment_seq_kernel(
    const uint8_t* __restrict__ src, const int64_t* __restrict__ idx, int V, int B, int H, int W,
    const float* __restrict__ lut, const float* __restrict__ recs, const uint32_t* __restrict__ gm,
    int gm_words, int group, unsigned long long seed, int order, Prog prog, TO* __restrict__ out) {
#pragma clang fp contract(off)
  __shared__ float s_img[kMaxHW];
  __shared__ float s_lut[256];
  const int rid = blockIdx.x;  // record = b * V + v
  const int b = rid / V, v = rid - b * V;
  const int HW = H * W;
  const float* rec = recs + (size_t)rid * AVD_AUG_REC;

  s_lut[threadIdx.x] = lut[threadIdx.x];
  __syncthreads();
  const uint32_t* row = reinterpret_cast<const uint32_t*>(src + (size_t)idx[b] * HW);
  for (int i = threadIdx.x; i < HW / 4; i += kThreads) {
    const uint32_t w4 = row[i];
    s_img[4 * i + 0] = s_lut[w4 & 0xFF];
    s_img[4 * i + 1] = s_lut[(w4 >> 8) & 0xFF];
    s_img[4 * i + 2] = s_lut[(w4 >> 16) & 0xFF];
    s_img[4 * i + 3] = s_lut[w4 >> 24];
  }
  __syncthreads();

  const int flags = (int)rec[AVD_AUG_FLAGS];
  View vw;               // the crop reads the current image
  vw.img = s_img;
  vw.H = H;
  vw.W = W;
  vw.crop = true;
  vw.top = (int)rec[AVD_AUG_CROP + 0];
  vw.left = (int)rec[AVD_AUG_CROP + 1];
  vw.ch = (int)rec[AVD_AUG_CROP + 2];
  vw.cw = (int)rec[AVD_AUG_CROP + 3];
  vw.sh = (float)vw.ch / (float)H;
  vw.sw = (float)vw.cw / (float)W;
  const float cx = (float)(W - 1) * 0.5f, cy = (float)(H - 1) * 0.5f;
  float acc[NPT];

  for (int s = 0; s < prog.n; ++s) {
    const int kind = prog.kind[s];
    bool gather = false;
    if (kind == SK_CROP) {
      if (!(flags & 1)) continue;
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const int p = threadIdx.x + k * kThreads;
        if (p < HW) {
          const int y = p / W;
          acc[k] = crop_sample(vw, y, p - y * W);
        }
      }
      gather = true;
    } else if (kind == SK_TWARP) {
      if (!(flags & 8)) continue;
      const float rate = rec[AVD_AUG_RATE];
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const int p = threadIdx.x + k * kThreads;
        if (p < HW) {
          const int y = p / W, x = p - y * W;
          const float t = (float)x * rate;
          float val = 0.0f;
          if (t < (float)W) {
            const int i0 = (int)t;
            const float a = t - (float)i0;
            const float s0 = fabsf(s_img[y * W + i0]);
            const float s1 = i0 + 1 < W ? fabsf(s_img[y * W + i0 + 1]) : 0.0f;
            val = a * s1 + (1.0f - a) * s0;
          }
          acc[k] = val;
        }
      }
      gather = true;
    } else if (kind == SK_ROT || kind == SK_AFF) {
      if (!(flags & (kind == SK_ROT ? 4 : 2))) continue;
      float m[6];
      const int o = kind == SK_ROT ? AVD_AUG_ROT : AVD_AUG_AFF;
#pragma unroll
      for (int j = 0; j < 6; ++j) m[j] = rec[o + j];
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const int p = threadIdx.x + k * kThreads;
        if (p < HW) {
          int qy = p / W, qx = p - qy * W;
          acc[k] = affine_nearest(m, cx, cy, W, H, qx, qy) ? s_img[qy * W + qx] : 0.0f;
        }
      }
      gather = true;
    } else if (kind == SK_FMASK || kind == SK_TMASK) {
      const int o = kind == SK_FMASK ? AVD_AUG_FMASK : AVD_AUG_TMASK;
      const int a0 = (int)rec[o], a1 = (int)rec[o + 1];
      if (a1 <= a0) continue;
      for (int p = threadIdx.x; p < HW; p += kThreads) {
        const int y = p / W, c = kind == SK_FMASK ? y : p - y * W;
        if (c >= a0 && c < a1) s_img[p] = 0.0f;
      }
    } else if (kind == SK_ERASE) {
      const int et = (int)rec[AVD_AUG_ERASE], el = (int)rec[AVD_AUG_ERASE + 1];
      const int eh = (int)rec[AVD_AUG_ERASE + 2], ew = (int)rec[AVD_AUG_ERASE + 3];
      if (eh <= 0) continue;
      for (int p = threadIdx.x; p < HW; p += kThreads) {
        const int y = p / W, x = p - y * W;
        if (y >= et && y < et + eh && x >= el && x < el + ew) s_img[p] = 0.0f;
      }
    } else if (kind == SK_NOISE) {
      const float nstd = rec[AVD_AUG_NOISE];
      if (nstd == 0.0f) continue;
      for (int q = threadIdx.x; q < HW / 2; q += kThreads) {
        const float2 g2 = gauss2(seed, (unsigned)rid, (unsigned)q);
        s_img[2 * q] = s_img[2 * q] + g2.x * nstd;
        s_img[2 * q + 1] = s_img[2 * q + 1] + g2.y * nstd;
      }
    } else if (kind == SK_GMASK) {
      const int gmrow = (int)rec[AVD_AUG_GM];
      if (!gm || gmrow < 0) continue;
      const uint32_t* gmr = gm + (size_t)gmrow * gm_words;
      const int gw = W / group;
      for (int p = threadIdx.x; p < HW; p += kThreads) {
        const int y = p / W, x = p - y * W;
        const int g = (y / group) * gw + x / group;
        if ((gmr[g >> 5] >> (g & 31)) & 1u) s_img[p] = s_img[p] * 0.0f;
      }
    } else {
      continue;
    }
    __syncthreads();      // every read of the previous image (gathers) / every update is done
    if (gather) {
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const int p = threadIdx.x + k * kThreads;
        if (p < HW) s_img[p] = acc[k];
      }
      __syncthreads();
    }
  }
  TO* o = out + (order == 0 ? (size_t)rid : (size_t)v * B + b) * HW;
  for (int q = threadIdx.x; q < HW / 2; q += kThreads) {
    if constexpr (sizeof(TO) == 4)
      reinterpret_cast<float2*>(o)[q] = make_float2(s_img[2 * q], s_img[2 * q + 1]);
    else
      reinterpret_cast<uint32_t*>(o)[q] = pack_bf16x2(s_img[2 * q], s_img[2 * q + 1]);
  }
}

// ----------------------------------------------------------------------------- parameter draws
// The chain's random parameters drawn on the device (what ViewAugmenter.records draws with
// numpy): one THREAD per (sample, view) record walks the stages in order with a counter-hash
// uniform stream (seed, record, draw index) -- records are independent, so a launch is n lanes
// of serial draws, not n blocks with one busy lane each; the grouped mask picks exactly k of the
// ng groups with Floyd's algorithm (a uniformly random k-subset, like randperm(ng)[:k]) on a
// per-thread bitmask in LDS.
struct Chain { float st[kMaxStages * kStageF]; int n; };

struct Urng {
  unsigned long long seed;
  unsigned rec, ctr;
  __device__ float u() {       // [0, 1), 24 bits
    const unsigned long long r = mix64(seed ^ mix64(((unsigned long long)rec << 32) | ctr++));
    return (float)(r >> 40) * 5.9604644775390625e-8f;
  }
  __device__ float uni(float a, float b) { return a + (b - a) * u(); }
  __device__ int below(int n) {  // uniform integer in [0, n)
    const int k = (int)(u() * (float)n);
    return k < n ? k : n - 1;
  }
};

// torchvision _get_inverse_affine_matrix, centre (0, 0), no shear
__device__ void inv_affine(float angle_deg, float tx, float ty, float s, float* m) {
  const float r = angle_deg * 0.017453292519943295f;
  const float c = cosf(r), sn = sinf(r);
  m[0] = c / s; m[1] = sn / s; m[2] = 0.f; m[3] = -sn / s; m[4] = c / s; m[5] = 0.f;
  m[2] += m[0] * (-tx) + m[1] * (-ty);
  m[5] += m[3] * (-tx) + m[4] * (-ty);
}

constexpr int kRecThreads = 64;

__global__ __launch_bounds__(kRecThreads) void aug_records_kernel(Chain ch, int n, int H, int W,
                                                                  int group,
                                                                  unsigned long long seed,
                                                                  float* __restrict__ recs,
                                                                  uint32_t* __restrict__ gm,
                                                                  int gm_words) {
  // the grouped-mask bitmask of each thread: word-major [word][thread] (conflict-free when the
  // lanes touch the same word index)
  __shared__ uint32_t bits[kMaxGroups / 32][kRecThreads];
  const int rid = blockIdx.x * kRecThreads + threadIdx.x;
  if (rid >= n) return;       // no barrier below: lanes are independent
  float* rec = recs + (size_t)rid * AVD_AUG_REC;
  Urng rng{seed, (unsigned)rid, 0u};
  float r[AVD_AUG_REC];
  for (int i = 0; i < AVD_AUG_REC; ++i) r[i] = 0.f;
  r[AVD_AUG_GM] = -1.f;
  int flags = 0, gk = -1, gon = 0;
  const float area = (float)(H * W);
  for (int si = 0; si < ch.n; ++si) {
    const float* a = ch.st + si * kStageF;
    const int kind = (int)a[0];
    const bool on = rng.u() < a[1];
    const float* q = a + 2;
    if (kind == SK_CROP || kind == SK_ERASE) {
      // RandomResizedCrop / RandomErasing get_params: 10 attempts, then the fallback
      const bool crop = kind == SK_CROP;
      const float l0 = logf(q[2]), l1 = logf(q[3]);
      int h = 0, w = 0, i = 0, j = 0;
      bool found = false;
      for (int t = 0; t < 10 && !found; ++t) {
        const float ta = area * rng.uni(q[0], q[1]);
        const float ar = expf(rng.uni(l0, l1));
        const int ww = (int)rintf(sqrtf(crop ? ta * ar : ta / ar));
        const int hh = (int)rintf(sqrtf(crop ? ta / ar : ta * ar));
        found = crop ? (ww > 0 && ww <= W && hh > 0 && hh <= H) : (hh < H && ww < W);
        if (found) { h = hh; w = ww; }
      }
      if (found) {
        i = rng.below(H - h + 1);
        j = rng.below(W - w + 1);
      } else if (crop) {      // centre crop at the nearest admissible aspect
        const float inr = (float)W / (float)H;
        if (inr < q[2]) { w = W; h = (int)rintf((float)W / q[2]); }
        else if (inr > q[3]) { h = H; w = (int)rintf((float)H * q[3]); }
        else { w = W; h = H; }
        i = (H - h) / 2;
        j = (W - w) / 2;
      }
      if (on) {
        const int o = crop ? AVD_AUG_CROP : AVD_AUG_ERASE;
        r[o] = (float)i; r[o + 1] = (float)j; r[o + 2] = (float)h; r[o + 3] = (float)w;
        if (crop) flags |= 1;
      }
    } else if (kind == SK_ROT) {
      float m[6];
      inv_affine(-rng.uni(-q[0], q[0]), 0.f, 0.f, 1.f, m);
      if (on) { for (int k = 0; k < 6; ++k) r[AVD_AUG_ROT + k] = m[k]; flags |= 4; }
    } else if (kind == SK_AFF) {
      const float ang = rng.uni(-q[0], q[0]);
      const float tx = q[1] >= 0.f ? rintf(rng.uni(-q[1] * W, q[1] * W)) : 0.f;
      const float ty = q[1] >= 0.f ? rintf(rng.uni(-q[2] * H, q[2] * H)) : 0.f;
      const float sc = q[3] > 0.f ? rng.uni(q[3], q[4]) : 1.f;
      float m[6];
      inv_affine(ang, tx, ty, sc, m);
      if (on) { for (int k = 0; k < 6; ++k) r[AVD_AUG_AFF + k] = m[k]; flags |= 2; }
    } else if (kind == SK_TWARP) {
      const float rate = rng.uni(q[0], q[1]);
      if (on) { r[AVD_AUG_RATE] = rate; flags |= 8; }
    } else if (kind == SK_FMASK || kind == SK_TMASK) {
      const int size = kind == SK_FMASK ? H : W;
      const float value = rng.u() * q[0];
      const float minv = rng.u() * ((float)size - value);
      const int st = (int)floorf(minv), en = st + (int)floorf(value);
      const int o = kind == SK_FMASK ? AVD_AUG_FMASK : AVD_AUG_TMASK;
      if (on) { r[o] = (float)st; r[o + 1] = (float)en; }
    } else if (kind == SK_NOISE) {
      if (on) r[AVD_AUG_NOISE] = q[0];
    } else if (kind == SK_GMASK) {
      const int ng = (H / group) * (W / group);
      gk = (int)(q[0] * (float)ng);
      gon = on;
      if (on) r[AVD_AUG_GM] = (float)rid;
    }
  }
  r[AVD_AUG_FLAGS] = (float)flags;
  for (int i = 0; i < AVD_AUG_REC; ++i) rec[i] = r[i];
  if (gk < 0 || !gm) return;
  // exactly k distinct groups (Floyd): for j = ng-k .. ng-1 draw t uniform in [0, j]; take t,
  // or j when t is taken already -- every k-subset equally likely
  const int ng = (H / group) * (W / group);
  const int words = (ng + 31) / 32;
  const int tx = threadIdx.x;
  for (int wd = 0; wd < words; ++wd) bits[wd][tx] = 0u;
  if (gon) {
    const unsigned long long key = (unsigned long long)(rid | 0x80000000u) << 32;
    for (int j = ng - gk; j < ng; ++j) {
      const unsigned h = (unsigned)(mix64(seed ^ mix64(key | (unsigned)j)) >> 32);
      const int t = (int)(((unsigned long long)h * (unsigned)(j + 1)) >> 32);   // [0, j]
      const bool taken = (bits[t >> 5][tx] >> (t & 31)) & 1u;
      const int g = taken ? j : t;
      bits[g >> 5][tx] |= 1u << (g & 31);
    }
  }
  uint32_t* row = gm + (size_t)rid * gm_words;
  for (int wd = 0; wd < gm_words; ++wd) row[wd] = wd < words ? bits[wd][tx] : 0u;
}

}  // namespace

extern "C" int avd_augment_views(const uint8_t* src_u8, const int64_t* idx, long long n_src, int B,
                                 int V, int H, int W, const float* lut, const float* rec,
                                 const uint32_t* gm, int gm_words, int group,
                                 unsigned long long seed, int order, float* out, void* stream) {
  if (!src_u8 || !idx || !lut || !rec || !out) return AVD_ERR_ARG;
  if (B <= 0 || V <= 0 || H <= 0 || W <= 0 || n_src <= 0) return AVD_ERR_SHAPE;
  if ((long long)H * W > kMaxHW || (H * W) % 4 || W % 2 || order < 0 || order > 1) return AVD_ERR_SHAPE;
  if (gm && (group <= 0 || H % group || W % group ||
             gm_words * 32 < (H / group) * (W / group)))
    return AVD_ERR_SHAPE;
  (void)n_src;  // sample ids are range-checked by the host wrapper (avdino.ops.augment_views)
  augment_kernel<float><<<B * V, kThreads, 0, avd_stream(stream)>>>(src_u8, idx, V, B, H, W, lut, rec, gm,
                                                                    gm_words, group, seed, order, out);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

extern "C" int avd_augment_views_dt(const uint8_t* src_u8, const int64_t* idx, long long n_src,
                                    int B, int V, int H, int W, const float* lut, const float* rec,
                                    const uint32_t* gm, int gm_words, int group,
                                    unsigned long long seed, int order, void* out, int odt,
                                    void* stream) {
  if (odt == AVD_F32)
    return avd_augment_views(src_u8, idx, n_src, B, V, H, W, lut, rec, gm, gm_words, group, seed,
                             order, (float*)out, stream);
  if (odt != AVD_BF16) return AVD_ERR_DTYPE;
  if (!src_u8 || !idx || !lut || !rec || !out) return AVD_ERR_ARG;
  if (B <= 0 || V <= 0 || H <= 0 || W <= 0 || n_src <= 0) return AVD_ERR_SHAPE;
  if ((long long)H * W > kMaxHW || (H * W) % 4 || W % 2 || order < 0 || order > 1) return AVD_ERR_SHAPE;
  if (gm && (group <= 0 || H % group || W % group ||
             gm_words * 32 < (H / group) * (W / group)))
    return AVD_ERR_SHAPE;
  augment_kernel<bf16><<<B * V, kThreads, 0, avd_stream(stream)>>>(src_u8, idx, V, B, H, W, lut, rec, gm,
                                                                   gm_words, group, seed, order,
                                                                   (bf16*)out);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

extern "C" int avd_augment_views_lds_check(const uint8_t* src_u8, const int64_t* idx, int B, int V,
                                           int H, int W, const float* lut, const float* rec,
                                           const uint32_t* gm, int gm_words, int group,
                                           unsigned long long seed, int order, void* out,
                                           int* chk, float* seen, void* stream) {
  if (!src_u8 || !idx || !lut || !rec || !out || !chk || !seen) return AVD_ERR_ARG;
  if (B <= 0 || V <= 0 || H <= 0 || W <= 0) return AVD_ERR_SHAPE;
  if ((long long)H * W > kMaxHW || (H * W) % 4 || W % 2 || order < 0 || order > 1) return AVD_ERR_SHAPE;
  if (gm && (group <= 0 || H % group || W % group || gm_words * 32 < (H / group) * (W / group)))
    return AVD_ERR_SHAPE;
  augment_kernel<bf16, true><<<B * V, kThreads, 0, avd_stream(stream)>>>(
      src_u8, idx, V, B, H, W, lut, rec, gm, gm_words, group, seed, order, (bf16*)out, chk, seen);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

// Diagnostic (tools/dbg_prefetch6.py): the gather kernel reading the source bytes and the byte
// table straight from global memory, no LDS (bf16 out)
extern "C" int avd_augment_views_nolds(const uint8_t* src_u8, const int64_t* idx, int B, int V, int H,
                                       int W, const float* lut, const float* rec, const uint32_t* gm,
                                       int gm_words, int group, unsigned long long seed, int order,
                                       void* out, void* stream) {
  if (!src_u8 || !idx || !lut || !rec || !out) return AVD_ERR_ARG;
  if (B <= 0 || V <= 0 || H <= 0 || W <= 0) return AVD_ERR_SHAPE;
  if ((long long)H * W > kMaxHW || (H * W) % 4 || W % 2 || order < 0 || order > 1) return AVD_ERR_SHAPE;
  if (gm && (group <= 0 || H % group || W % group || gm_words * 32 < (H / group) * (W / group)))
    return AVD_ERR_SHAPE;
  augment_kernel<bf16, false, true><<<B * V, kThreads, 0, avd_stream(stream)>>>(
      src_u8, idx, V, B, H, W, lut, rec, gm, gm_words, group, seed, order, (bf16*)out);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

extern "C" int avd_augment_views_seq(const uint8_t* src_u8, const int64_t* idx, long long n_src,
                                     int B, int V, int H, int W, const float* lut, const float* rec,
                                     const uint32_t* gm, int gm_words, int group,
                                     unsigned long long seed, int order, const int* kinds,
                                     int nkinds, void* out, int odt, void* stream) {
  if (!src_u8 || !idx || !lut || !rec || !out || (nkinds > 0 && !kinds)) return AVD_ERR_ARG;
  if (B <= 0 || V <= 0 || H <= 0 || W <= 0 || n_src <= 0) return AVD_ERR_SHAPE;
  if ((long long)H * W > kMaxHW || (H * W) % 4 || W % 2 || order < 0 || order > 1) return AVD_ERR_SHAPE;
  if (nkinds < 0 || nkinds > kMaxStages) return AVD_ERR_SHAPE;
  Prog prog{};
  prog.n = nkinds;
  bool has_gm = false;
  for (int i = 0; i < nkinds; ++i) {
    if (kinds[i] < SK_CROP || kinds[i] > SK_GMASK) return AVD_ERR_ARG;
    prog.kind[i] = kinds[i];
    has_gm |= kinds[i] == SK_GMASK;
  }
  if (gm && has_gm && (group <= 0 || H % group || W % group ||
                       gm_words * 32 < (H / group) * (W / group)))
    return AVD_ERR_SHAPE;
  if (odt != AVD_F32 && odt != AVD_BF16) return AVD_ERR_DTYPE;
  const int npt = avd_cdiv(H * W, kThreads);
  hipStream_t st = avd_stream(stream);
#define AVD_SEQ_LAUNCH(TO, N)                                                                  \
  augment_seq_kernel<TO, N><<<B * V, kThreads, 0, st>>>(src_u8, idx, V, B, H, W, lut, rec, gm,  \
                                                        gm_words, group, seed, order, prog,     \
                                                        (TO*)out)
  if (npt <= 4) {
    if (odt == AVD_F32) AVD_SEQ_LAUNCH(float, 4); else AVD_SEQ_LAUNCH(bf16, 4);
  } else if (npt <= 16) {
    if (odt == AVD_F32) AVD_SEQ_LAUNCH(float, 16); else AVD_SEQ_LAUNCH(bf16, 16);
  } else {
    if (odt == AVD_F32) AVD_SEQ_LAUNCH(float, 49); else AVD_SEQ_LAUNCH(bf16, 49);
  }
#undef AVD_SEQ_LAUNCH
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

extern "C" int avd_augment_records(const float* stages, int nstages, int n, int H, int W,
                                   int group, unsigned long long seed, float* rec, uint32_t* gm,
                                   int gm_words, void* stream) {
  if (!stages || !rec) return AVD_ERR_ARG;
  if (nstages < 0 || nstages > kMaxStages || n <= 0 || H <= 0 || W <= 0) return AVD_ERR_SHAPE;
  Chain ch{};
  ch.n = nstages;
  bool has_gm = false;
  for (int i = 0; i < nstages * kStageF; ++i) ch.st[i] = stages[i];
  for (int i = 0; i < nstages; ++i) has_gm |= (int)stages[i * kStageF] == SK_GMASK;
  if (has_gm) {
    if (!gm || group <= 0 || H % group || W % group) return AVD_ERR_SHAPE;
    const int ng = (H / group) * (W / group);
    if (ng > kMaxGroups || gm_words * 32 < ng) return AVD_ERR_SHAPE;
  }
  aug_records_kernel<<<avd_cdiv(n, kRecThreads), kRecThreads, 0, avd_stream(stream)>>>(
      ch, n, H, W, group, seed, rec, has_gm ? gm : nullptr, gm_words);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}
