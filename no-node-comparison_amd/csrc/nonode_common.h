// nonode_common.h — declarations shared by the library's translation units (nonode.hip and
// nonode_node.hip): the vector types, the packed layer-blob layout, the launch utilities and the
// device helpers (ECL layout, f32 and fp16x3 MFMA products). Everything is internal to each unit
// (anonymous namespace) except the error string, which is one per library.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "nonode.h"

namespace nonode_tu {
extern thread_local std::string g_err;   // nonode_last_error(); defined in nonode.hip
}

namespace {

using nonode_tu::g_err;

typedef float f4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f8 __attribute__((ext_vector_type(8)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));

constexpr int HID = 64;    // hidden width (hidden_nf in model_confs.yaml:5,25)
constexpr int ROWP = 68;   // LDS row stride of node tables (floats): 64 + 4 breaks bank aliasing
constexpr int TMAX = 16;   // max trajectory length handled by tconv_kernel
constexpr int MMAX = 9;    // max Fourier modes (T <= 16: at most T/2 + 1 = 9 rfft bins)

// ---- packed layer blob (floats) --------------------------------------------------------------
// Fragment matrices: W[64][I] used as the A operand of v_mfma_f32_16x16x4_f32 with the B operand
// in the "edge-column layout" (ECL): lane l = 16*g + e holds, for channel group mt and q in 0..3,
// channel 16*mt + 4*g + q of column e. frag(mo, mt)[lane][q] = W[16*mo + (l&15)][16*mt + 4*(l>>4) + q]
// so one MFMA's output accumulator IS the next MFMA's B operand (no lane movement).
enum : int {
  OFF_WA = 0,        // edge W1 h_i columns  [64x64]
  OFF_WB = 4096,     // edge W1 h_j columns  [64x64]
  OFF_W2 = 8192,     // edge W2              [64x64]
  OFF_WC1 = 12288,   // coord W1             [64x64]
  OFF_WV1 = 16384,   // node_v W1            [64x64] (EGNO)
  OFF_WN1 = 20480,   // node W1              [64x128]
  OFF_WN2 = 28672,   // node W2              [64x64]
  OFF_FEAT = 32768,  // edge W1 columns of the scalar edge inputs [|r|^2, e_0 .. e_{ne-1}] as up to
                     // two extra k-steps: feat[kf][lane][mo] = W1[16*mo + (l&15)][feature 4*kf + (l>>4)]
  OFF_VEC = 33280,   // vectors, 64 floats each, in "vp" order vp[16*g + 4*mt + q] = v[16*mt + 4*g + q]
  OFF_H16 = 33856,   // W2 | Wc1 as fp16 hi/lo fragments of v_mfma_f32_16x16x32_f16 (2 x 4096 floats):
                     // [mat][s][mo][hi|lo][lane][8 halves], half j of lane l = W[16*mo + (l&15)][chan(s, l>>4, j)],
                     // chan(s, g, j) = 16*(2*s + (j>>2)) + 4*g + (j&3)  (the ECL order, see h16_b)
  OFF_H16N = 33856 + 8192,   // node-side matrices in the same fp16 hi/lo layout, 4096 floats each (H_*)
};
enum : int { H_WA = 0, H_WB, H_WV1, H_WN1A, H_WN1B, H_WN2, H_COUNT };   // WN1A/B: h / message-sum columns
enum : int { V_B2 = 0, V_BC1, V_WC2, V_B1, V_BV1, V_WV2, V_BN1, V_BN2, V_COUNT };
constexpr int OFF_SCAL = OFF_VEC + V_COUNT * 64;  // [0] = coord b2, [1] = node_v b2, [SC_*] option flags
// option flags (1.f / 0.f): radial input normalised (EGNO norm=True, basic.py:140-141); coordinate
// MLP output through tanh (SEGNO tanh=True, gcl.py:57-59)
constexpr int SC_NORM = 2, SC_TANH = 3;
// packed half2 lo-part shifts of the fp16x3 matrices (h8_scale): slots SC_H16S + HS_*
constexpr int SC_H16S = 8;
enum : int { HS_W2 = 0, HS_WC1 = 1, HS_N = 2, HS_COUNT = HS_N + 6 };   // HS_N + H_*: node-side matrices
// F.normalize of the one-element radial feature: s / max(|s|, 1e-12) (s >= 0: 1 unless s < 1e-12)
// (inf, NaN -> NaN as inf / inf and NaN / NaN in the reference)
__device__ __forceinline__ float radial_norm(float s) {
  return s < 1e-12f ? s * 1e12f : (__builtin_isfinite(s) ? 1.f : s - s);
}
static_assert(OFF_SCAL + 64 == OFF_H16, "blob layout");
constexpr int BLOB_FLOATS = OFF_H16N + H_COUNT * 4096;
constexpr float H16_LIMIT = 16384.f;   // |activation| above this takes the exact f32 MFMA path
constexpr int EDGE_STAGE_FLOATS = 512 + 3 * 64;   // FEAT | b2 | bc1 | wc2 (contiguous) staged to LDS


int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(NONODE_ELAUNCH, "%s: %s", what, hipGetErrorString(e));
  return NONODE_OK;
}

int num_cus() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cache[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    cache[dev] = n;
  }
  return cache[dev];
}

// ---- device helpers ---------------------------------------------------------------------------
// SiLU in the log2 domain. Every SiLU input z is produced by a packed linear layer whose weights
// and bias were pre-multiplied by -log2(e) (pack_kernel), so the kernel sees z' = -log2(e) z and
//   silu2(z') = z' / (1 + 2^z') = -log2(e) * SiLU(z)
// (v_exp_f32 + v_add + v_rcp + v_mul: the multiply of __expf is gone). The -ln 2 that undoes the
// factor is folded into whatever consumes the output: the next layer's weights (where it cancels
// against the next -log2(e)), the coord / node_v output vectors, and node W2.
__device__ __forceinline__ float silu(float z) {
  return z * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(z));
}
constexpr float NEG_LOG2E = -1.4426950408889634f;   // scale of every SiLU input
constexpr float NEG_LN2 = -0.6931471805599453f;     // 1 / NEG_LOG2E, scale of every SiLU consumer

__device__ __forceinline__ f4 mfma(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// acc[mo] += sum over the KT*16 input channels of W frag(mo, .) * in (ECL); wf = blob section.
// acc[mo] += sum over the KT*16 input channels of W frag(mo, .) * in (ECL); wf = blob section.
// Fully unrolled (static register indexing); fragments of step mt+1 are loaded while the 16 MFMAs
// of step mt issue, and a scheduling barrier per step keeps at most two steps of fragments live.
template <int KT>
__device__ __forceinline__ void mfma_dense(f4 (&acc)[4], const float* __restrict__ wf, const f4* in,
                                           int lane) {
  f4 a[2][4];
#pragma unroll
  for (int mo = 0; mo < 4; ++mo) a[0][mo] = *reinterpret_cast<const f4*>(wf + ((mo * KT + 0) * 64 + lane) * 4);
#pragma unroll
  for (int mt = 0; mt < KT; ++mt) {
    if (mt + 1 < KT) {
#pragma unroll
      for (int mo = 0; mo < 4; ++mo)
        a[(mt + 1) & 1][mo] = *reinterpret_cast<const f4*>(wf + ((mo * KT + mt + 1) * 64 + lane) * 4);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int mo = 0; mo < 4; ++mo) acc[mo] = mfma(a[mt & 1][mo][q], in[mt][q], acc[mo]);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Two independent column sets (two edge units) through the same weights: each fragment read
// feeds two MFMAs, and the 8 accumulator chains hide the MFMA dependency latency.
template <int KT>
__device__ __forceinline__ void mfma_dense2(f4 (&acc0)[4], f4 (&acc1)[4], const float* __restrict__ wf,
                                            const f4* in0, const f4* in1, int lane) {
  f4 a[2][4];
#pragma unroll
  for (int mo = 0; mo < 4; ++mo) a[0][mo] = *reinterpret_cast<const f4*>(wf + ((mo * KT + 0) * 64 + lane) * 4);
#pragma unroll
  for (int mt = 0; mt < KT; ++mt) {
    if (mt + 1 < KT) {
#pragma unroll
      for (int mo = 0; mo < 4; ++mo)
        a[(mt + 1) & 1][mo] = *reinterpret_cast<const f4*>(wf + ((mo * KT + mt + 1) * 64 + lane) * 4);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int mo = 0; mo < 4; ++mo) {
        acc0[mo] = mfma(a[mt & 1][mo][q], in0[mt][q], acc0[mo]);
        acc1[mo] = mfma(a[mt & 1][mo][q], in1[mt][q], acc1[mo]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

__device__ __forceinline__ void load_frags(f4 (&a)[4], const float* wf, int mt, int lane) {
#pragma unroll
  for (int mo = 0; mo < 4; ++mo) a[mo] = *reinterpret_cast<const f4*>(wf + ((mo * 4 + mt) * 64 + lane) * 4);
}

// ---- fp16x3 split MFMA (fp32-level accuracy at fp16 matrix-core rate) ------------------------
// x = hi + lo with hi = fp16(x), lo = fp16(x - hi): |x - hi - lo| <= 2^-22 |x| while lo is an fp16
// normal, i.e. for |x| >= ~2^-3; below that lo is subnormal and the split error is the absolute
// 2^-25 of the fp16 subnormal spacing. Weights take a per-matrix power-of-two shift of their lo part
// for this reason (h8_scale below); activations are O(1) SiLU outputs / states. W x is accumulated
// in fp32 as W_hi x_hi + W_lo x_hi + W_hi x_lo (the dropped W_lo x_lo term is ~2^-22 relative); the
// chain starts with the product that needs only the hi conversions, so the residual and the x_hi''
// scaling of the other two terms issue under its MFMAs.
// The ECL accumulator of one layer is the B operand of v_mfma_f32_16x16x32_f16 for the next:
// k-step s, half j of lane (g, e) = channel 16*(2s + (j>>2)) + 4g + (j&3) of column e.
// x - (float)half(hp): one v_fma_mix_f32 (f16 operand taken from the low / high half of hp). For
// |x| in the fp16 range the difference is exactly representable, so the residual is exact.
// The asm writes its result over x's own register ("+v"): that register was last written by a
// compiler-visible VALU instruction (x's producer, or a copy of x the compiler makes when x stays live),
// which already met every MFMA hazard. A fresh "=v" output could be a register that an MFMA issued
// just before still reads as SrcC, and the hazard recognizer does not treat an asm block as a VALU
// write, so it would not pad that WAR hazard.
__device__ __forceinline__ float resid_lo(unsigned hp, float x) {
  asm("v_fma_mix_f32 %0, -%1, 1.0, %0 op_sel_hi:[1,0,0]" : "+v"(x) : "v"(hp));
  return x;
}
__device__ __forceinline__ float resid_hi(unsigned hp, float x) {
  asm("v_fma_mix_f32 %0, -%1, 1.0, %0 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(x) : "v"(hp));
  return x;
}
__device__ __forceinline__ void h16_split(const f4 (&x)[4], h8 (&hi)[2], h8 (&lo)[2]) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const f8 v = {x[2 * s][0], x[2 * s][1], x[2 * s][2], x[2 * s][3],
                  x[2 * s + 1][0], x[2 * s + 1][1], x[2 * s + 1][2], x[2 * s + 1][3]};
    hi[s] = __builtin_convertvector(v, h8);                       // v_cvt_pk_f16_f32 (RNE)
    const auto hw = __builtin_bit_cast(u4, hi[s]);
    f8 r;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      r[2 * i] = resid_lo(hw[i], v[2 * i]);
      r[2 * i + 1] = resid_hi(hw[i], v[2 * i + 1]);
    }
    lo[s] = __builtin_convertvector(r, h8);
  }
}
__device__ __forceinline__ float amax_ecl(const f4 (&x)[4]) {
  float m = 0.f;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int q = 0; q < 4; ++q) m = fmaxf(m, fabsf(x[mt][q]));
  return m;
}
__device__ __forceinline__ f4 mfma16(h8 a, h8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
// The weight residual W_lo = W - W_hi is ~2^-11 |W|: for |W| < 2^-3 it would be an fp16 subnormal
// with a 2^-25 absolute floor (3e-5 relative at |W| = 2^-10). So each packed 64x64 matrix stores
// W_lo' = 2^k W_lo, k the per-matrix shift that puts max |W| 2^k in [2^H16_LO_TARGET, 2^(T+1)), and the
// kernels pair it with x_hi'' = 2^-k x_hi (one v_pk_mul_f16 per two halves; exact while x_hi'' is an
// fp16 normal, and a subnormal x_hi'' only touches the ~2^-11 correction term): W_lo x_hi = W_lo' x_hi''.
// `us` is the packed half2 (2^-k, 2^-k) of the matrix (blob OFF_SCAL + SC_H16S + index).
// (a compiler-visible multiply, not inline asm: the hazard recognizer does not see an asm VALU
// write, so an MFMA could read its result, or an asm could overwrite a pending MFMA's operand,
// without the required wait states)
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ h8 h8_scale(h8 x, unsigned us) {
  const h2 sc = __builtin_bit_cast(h2, us);
  const u4 w = __builtin_bit_cast(u4, x);
  u4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const unsigned wi = w[i];   // (an rvalue: __builtin_bit_cast of a vector element reads element 0)
    r[i] = __builtin_bit_cast(unsigned, __builtin_bit_cast(h2, wi) * sc);
  }
  return __builtin_bit_cast(h8, r);
}
// one edge unit through one 64x64 layer: acc += W x (24 MFMAs, 4 chains)
__device__ __forceinline__ void mfma_h16(f4 (&acc)[4], const h8* wf, const h8 (&xh)[2], const h8 (&xl)[2],
                                         int lane, unsigned us) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    h8 ah[4], al[4];
#pragma unroll
    for (int mo = 0; mo < 4; ++mo) {
      ah[mo] = wf[((s * 4 + mo) * 2 + 0) * 64 + lane];
      al[mo] = wf[((s * 4 + mo) * 2 + 1) * 64 + lane];
    }
    const h8 xs = h8_scale(xh[s], us);
#pragma unroll
    for (int mo = 0; mo < 4; ++mo) acc[mo] = mfma16(ah[mo], xh[s], acc[mo]);
#pragma unroll
    for (int mo = 0; mo < 4; ++mo) acc[mo] = mfma16(al[mo], xs, acc[mo]);
#pragma unroll
    for (int mo = 0; mo < 4; ++mo) acc[mo] = mfma16(ah[mo], xl[s], acc[mo]);
  }
}

// acc += W x for one 16-column tile: fp16x3 on the matrix cores, or the exact f32 MFMA path (wf)
// when any |x| is beyond the fp16 hi range (wave-uniform guard)
__device__ __forceinline__ void mm64(f4 (&acc)[4], const h8* wh, const float* wf, const f4 (&x)[4], int lane,
                                     unsigned us) {
  if (__builtin_expect(__any(amax_ecl(x) > H16_LIMIT), 0)) {
    mfma_dense<4>(acc, wf, x, lane);
  } else {
    h8 xh[2], xl[2];
    h16_split(x, xh, xl);
    mfma_h16(acc, wh, xh, xl, lane, us);
  }
}

// Fragments of one 64x64 matrix held in registers: [s][mo] hi and lo (64 VGPRs).
struct H16Frags {
  h8 hi[2][4], lo[2][4];
};
__device__ __forceinline__ void load_h16frags(H16Frags& f, const h8* wf, int lane) {
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int mo = 0; mo < 4; ++mo) {
      f.hi[s][mo] = wf[((s * 4 + mo) * 2 + 0) * 64 + lane];
      f.lo[s][mo] = wf[((s * 4 + mo) * 2 + 1) * 64 + lane];
    }
}
// keep fragments in AGPRs: the MFMAs read them as their A operand directly (a plain hoist leaves
// them in AGPRs too, but copies them back with v_accvgpr_read before every use)
__device__ __forceinline__ void pin_agpr(H16Frags& f) {
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int mo = 0; mo < 4; ++mo) {
      asm volatile("" : "+a"(f.hi[s][mo]));
      asm volatile("" : "+a"(f.lo[s][mo]));
    }
}
// two edge units through register-resident fragments, the two chains interleaved
__device__ __forceinline__ void mfma_h16r2(f4 (&acc0)[4], f4 (&acc1)[4], const H16Frags& f, const h8 (&x0h)[2],
                                           const h8 (&x0l)[2], const h8 (&x1h)[2], const h8 (&x1l)[2], unsigned us) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const h8 x0s = h8_scale(x0h[s], us), x1s = h8_scale(x1h[s], us);
#pragma unroll
    for (int mo = 0; mo < 4; ++mo) { acc0[mo] = mfma16(f.hi[s][mo], x0h[s], acc0[mo]); acc1[mo] = mfma16(f.hi[s][mo], x1h[s], acc1[mo]); }
#pragma unroll
    for (int mo = 0; mo < 4; ++mo) { acc0[mo] = mfma16(f.lo[s][mo], x0s, acc0[mo]); acc1[mo] = mfma16(f.lo[s][mo], x1s, acc1[mo]); }
#pragma unroll
    for (int mo = 0; mo < 4; ++mo) { acc0[mo] = mfma16(f.hi[s][mo], x0l[s], acc0[mo]); acc1[mo] = mfma16(f.hi[s][mo], x1l[s], acc1[mo]); }
  }
}

// three edge units through register-resident fragments (the triple loop, NONODE_TRIPLE builds)
__device__ __forceinline__ void mfma_h16r3(f4 (&acc0)[4], f4 (&acc1)[4], f4 (&acc2)[4], const H16Frags& f,
                                           const h8 (&x0h)[2], const h8 (&x0l)[2], const h8 (&x1h)[2],
                                           const h8 (&x1l)[2], const h8 (&x2h)[2], const h8 (&x2l)[2], unsigned us) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const h8 x0s = h8_scale(x0h[s], us), x1s = h8_scale(x1h[s], us), x2s = h8_scale(x2h[s], us);
#pragma unroll
    for (int mo = 0; mo < 4; ++mo) {
      acc0[mo] = mfma16(f.hi[s][mo], x0h[s], acc0[mo]);
      acc1[mo] = mfma16(f.hi[s][mo], x1h[s], acc1[mo]);
      acc2[mo] = mfma16(f.hi[s][mo], x2h[s], acc2[mo]);
    }
#pragma unroll
    for (int mo = 0; mo < 4; ++mo) {
      acc0[mo] = mfma16(f.lo[s][mo], x0s, acc0[mo]);
      acc1[mo] = mfma16(f.lo[s][mo], x1s, acc1[mo]);
      acc2[mo] = mfma16(f.lo[s][mo], x2s, acc2[mo]);
    }
#pragma unroll
    for (int mo = 0; mo < 4; ++mo) {
      acc0[mo] = mfma16(f.hi[s][mo], x0l[s], acc0[mo]);
      acc1[mo] = mfma16(f.hi[s][mo], x1l[s], acc1[mo]);
      acc2[mo] = mfma16(f.hi[s][mo], x2l[s], acc2[mo]);
    }
  }
}

// two units (or tiles) through one fp16x3 matrix read from LDS or L2: each fragment read feeds both
// units' MFMAs, and each accumulator sees the same MFMA sequence as mfma_h16 (bitwise the same sums)
__device__ __forceinline__ void mfma_h16x2(f4 (&acc0)[4], f4 (&acc1)[4], const h8* wf, const h8 (&x0h)[2],
                                           const h8 (&x0l)[2], const h8 (&x1h)[2], const h8 (&x1l)[2], int lane,
                                           unsigned us) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    h8 ah[4], al[4];
#pragma unroll
    for (int mo = 0; mo < 4; ++mo) {
      ah[mo] = wf[((s * 4 + mo) * 2 + 0) * 64 + lane];
      al[mo] = wf[((s * 4 + mo) * 2 + 1) * 64 + lane];
    }
    const h8 x0s = h8_scale(x0h[s], us), x1s = h8_scale(x1h[s], us);
#pragma unroll
    for (int mo = 0; mo < 4; ++mo) { acc0[mo] = mfma16(ah[mo], x0h[s], acc0[mo]); acc1[mo] = mfma16(ah[mo], x1h[s], acc1[mo]); }
#pragma unroll
    for (int mo = 0; mo < 4; ++mo) { acc0[mo] = mfma16(al[mo], x0s, acc0[mo]); acc1[mo] = mfma16(al[mo], x1s, acc1[mo]); }
#pragma unroll
    for (int mo = 0; mo < 4; ++mo) { acc0[mo] = mfma16(ah[mo], x0l[s], acc0[mo]); acc1[mo] = mfma16(ah[mo], x1l[s], acc1[mo]); }
  }
}
// mm64 for two tiles: the fp16x3 path shares every fragment read between them. The range guard stays
// per tile (a tile past the fp16 hi range takes mm64's exact f32 path, and so, in that rare case, does
// its partner through its own mm64), so each tile's result is bitwise mm64's.
__device__ __forceinline__ void mm64x2(f4 (&acc0)[4], f4 (&acc1)[4], const h8* wh, const float* wf, const f4 (&x0)[4],
                                       const f4 (&x1)[4], int lane, unsigned us) {
  if (__builtin_expect(__any(fmaxf(amax_ecl(x0), amax_ecl(x1)) > H16_LIMIT), 0)) {
    mm64(acc0, wh, wf, x0, lane, us);
    mm64(acc1, wh, wf, x1, lane, us);
  } else {
    h8 x0h[2], x0l[2], x1h[2], x1l[2];
    h16_split(x0, x0h, x0l);
    h16_split(x1, x1h, x1l);
    mfma_h16x2(acc0, acc1, wh, x0h, x0l, x1h, x1l, lane, us);
  }
}

// f4 sum as four plain v_add_f32: the backend would emit two v_pk_add_f32, which cost more than the
// plain ops they replace when issued beside MFMAs (MI355X_MICROARCH.md constants table)
__device__ __forceinline__ f4 add4(f4 a, f4 b) {
  f4 r;
#pragma unroll
  for (int q = 0; q < 4; ++q) {   // in place, for the reason given at resid_lo
    r[q] = a[q];
    asm("v_add_f32 %0, %0, %1" : "+v"(r[q]) : "v"(b[q]));
  }
  return r;
}
__device__ __forceinline__ void load_ecl(f4 (&d)[4], const float* row, int g) {
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) d[mt] = *reinterpret_cast<const f4*>(row + 16 * mt + 4 * g);
}
__device__ __forceinline__ void store_ecl(float* row, const f4 (&s)[4], int g) {
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) *reinterpret_cast<f4*>(row + 16 * mt + 4 * g) = s[mt];
}
// vector in vp order: lane group g reads its 16 channels as 4 float4
__device__ __forceinline__ void load_vp(f4 (&d)[4], const float* vp, int g) {
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) d[mt] = *reinterpret_cast<const f4*>(vp + 16 * g + 4 * mt);
}
// SiLU of the 16 ECL values (plain f32 add / multiply: packed v_pk_* ops issued beside the MFMAs
// measured 1.8% slower, C2 layer 252 vs 247.5 us)
__device__ __forceinline__ void silu_ecl(f4 (&a)[4]) {
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int q = 0; q < 4; ++q) a[mt][q] = silu(a[mt][q]);
}
// sum over the 4 lane groups (lanes e, e+16, e+32, e+48): the full 64-channel dot product
// (gfx950 permlane swaps: v + v^32 and then v + v^16 without an LDS round trip)
__device__ __forceinline__ float group_sum(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
__device__ __forceinline__ float dot_r(const f4 (&a)[4], const f4 (&w)[4]) {
  float s = 0.f;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int q = 0; q < 4; ++q) s = fmaf(a[mt][q], w[mt][q], s);
  return group_sum(s);
}
__device__ __forceinline__ float dot_vp(const f4 (&a)[4], const float* vp, int g) {
  f4 w[4];
  load_vp(w, vp, g);
  float s = 0.f;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int q = 0; q < 4; ++q) s = fmaf(a[mt][q], w[mt][q], s);
  return group_sum(s);
}

// sum over the P lane groups of 16 / P columns inside each 16-lane row (P = 2: lanes e, e +- 8;
// P = 4: e, e +- 4, e +- 8, e +- 12), by DPP row rotations in a fixed order (column packing of the
// layer kernel's last tile)
template <int R>
__device__ __forceinline__ float row_ror(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x120 + R, 0xF, 0xF, false));
}
__device__ __forceinline__ float group_fold(float v, int P) {
  if (P == 4) v += row_ror<4>(v);
  return v + row_ror<8>(v);
}

// ---- balanced split of a chunk's edge units over the waves (pair mode) ----------------------------
// A wave's range is walked tile segment by tile segment: per segment a fixed cost (tile state,
// fragment loads, the flush), then pairs of units up to the tile's packed limit Q and single units
// after (the pair loop's odd unit, a packed tile's regular units). Modelled costs (stamped, C3:
// ~3.2K cycles per segment, ~6.4K per pair or single on average):
constexpr int CS_SEG = 2, CS_PAIR = 4, CS_ONE = 3;
// cost of units k..kend (1-based offsets) of a tile with packed limit Q
__device__ __forceinline__ int seg_cost(int k, int kend, int Q) {
  const int lp = max(min(kend, Q) - k + 1, 0), lr = max(kend - max(k, Q + 1) + 1, 0);
  return CS_SEG + CS_PAIR * (lp >> 1) + CS_ONE * ((lp & 1) + lr);
}
// the most units from offset k on (tile of L units, packed limit Q) within budget b
__device__ __forceinline__ int seg_take(int k, int L, int Q, int b) {
  int bb = b - CS_SEG;
  if (bb < CS_ONE) return 0;
  const int lp = max(Q - k + 1, 0);
  const int np = bb / CS_PAIR;
  if (2 * np < lp) return 2 * np + (bb - CS_PAIR * np >= CS_ONE ? 1 : 0);
  bb -= CS_PAIR * (lp >> 1) + CS_ONE * (lp & 1);
  return lp + min(L - max(k, Q + 1) + 1, bb / CS_ONE);
}
// Contiguous ranges of the U = (ctc - 1) Nm1 + Ul units (last tile: Ul units, packed limit Ql) over
// NW waves with the smallest modelled maximum (binary search on it, greedy fill). Wave w takes units
// [cut[w], cut[w + 1]). Returns whether budget T fits (cut then holds the fill).
// (cut: this wave's own LDS copy: every lane writes the same values)
template <int NW>
__device__ __forceinline__ bool unit_fill(int T, int ctc, int Nm1, int Ul, int Ql, int* cut) {
  int w = 0, b = T, t = 0, k = 1;
  const int U = (ctc - 1) * Nm1 + Ul;
  cut[0] = 0;
  while (t < ctc) {
    const int L = t == ctc - 1 ? Ul : Nm1, Q = t == ctc - 1 ? Ql : Nm1;
    const int n = seg_take(k, L, Q, b);
    if (k + n - 1 == L) {
      b -= seg_cost(k, L, Q);
      ++t;
      k = 1;
    } else {
      k += n;
      if (++w == NW) return false;
      b = T;
      cut[w] = t * Nm1 + k - 1;
    }
  }
  for (int i = w + 1; i <= NW; ++i) cut[i] = U;
  return true;
}
template <int NW>
__device__ __forceinline__ void unit_split(int ctc, int Nm1, int Ul, int Ql, int* cut) {
  int lo = 0, hi = 0;
  for (int t = 0; t < ctc; ++t) hi += seg_cost(1, t == ctc - 1 ? Ul : Nm1, t == ctc - 1 ? Ql : Nm1);
  while (lo < hi) {   // smallest T that fits
    const int mid = (lo + hi) >> 1;
    if (unit_fill<NW>(mid, ctc, Nm1, Ul, Ql, cut)) hi = mid;
    else lo = mid + 1;
  }
  unit_fill<NW>(lo, ctc, Nm1, Ul, Ql, cut);
}
// max over the 4 lane groups (the column max of an ECL activation)
__device__ __forceinline__ float group_max(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
// acc = W x + bias for one 16-column unit whose activations may leave the fp16 range (the guard
// path): every column (edge) is scaled by 2^-s, s >= 0 the smallest shift that brings its largest
// |value| below 2^13, before the fp16x3 split, and the product is scaled back by 2^s. Both scalings
// are exact; the split is then ~2^-22 relative to each column's largest |value| (not to each element:
// elements more than ~2^16 below their column's maximum fall into the fp16 subnormal range).
// the same with the fragments in registers (the pair loop's AGPR-resident W2 / Wc1)
__device__ __forceinline__ void mm64_scaled(f4 (&acc)[4], const H16Frags& f, const f4 (&x)[4], unsigned us) {
  const float cmax = group_max(amax_ecl(x));
  const int s = max(__builtin_amdgcn_frexp_expf(cmax) - 13, 0);
  const float dn = __uint_as_float((unsigned)(127 - s) << 23), up = __uint_as_float((unsigned)(127 + min(s, 127)) << 23);
  f4 xs[4], t[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) { xs[mt] = x[mt] * dn; t[mt] = f4{0.f, 0.f, 0.f, 0.f}; }
  h8 xh[2], xl[2];
  h16_split(xs, xh, xl);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const h8 xs2 = h8_scale(xh[k], us);
#pragma unroll
    for (int mo = 0; mo < 4; ++mo) t[mo] = mfma16(f.hi[k][mo], xh[k], t[mo]);
#pragma unroll
    for (int mo = 0; mo < 4; ++mo) t[mo] = mfma16(f.lo[k][mo], xs2, t[mo]);
#pragma unroll
    for (int mo = 0; mo < 4; ++mo) t[mo] = mfma16(f.hi[k][mo], xl[k], t[mo]);
  }
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) acc[mt] += t[mt] * up;
}
__device__ __forceinline__ void mm64_scaled(f4 (&acc)[4], const h8* wh, const f4 (&x)[4], int lane, unsigned us) {
  const float cmax = group_max(amax_ecl(x));
  const int s = max(__builtin_amdgcn_frexp_expf(cmax) - 13, 0);
  const float dn = __uint_as_float((unsigned)(127 - s) << 23), up = __uint_as_float((unsigned)(127 + min(s, 127)) << 23);
  f4 xs[4], t[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) { xs[mt] = x[mt] * dn; t[mt] = f4{0.f, 0.f, 0.f, 0.f}; }
  h8 xh[2], xl[2];
  h16_split(xs, xh, xl);
  mfma_h16(t, wh, xh, xl, lane, us);
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) acc[mt] += t[mt] * up;
}

// packed half2 (2^-k, 2^-k) of an fp16x3 matrix (blob scalar slot SC_H16S + idx, see h8_scale)
__device__ __forceinline__ unsigned h16_us(const float* scal, int idx) {
  return __float_as_uint(scal[SC_H16S + idx]);
}

}  // namespace
