// nonode_tconv.hip — the TimeConv reverse (layer_no.py:80-126 reversed; oracle/egno_grad.py
// spectral_bwd), its own translation unit: built with the default machine scheduler and MFMA
// accumulators in AGPRs (LLVM's AGPR-copy rewrite of the VGPR-form build crashes on the higher-mode
// instances, and the three-group two-mode instance keeps its accumulators out of the 170 registers of
// a three-waves-per-SIMD workgroup).
#include "nonode_bwd_common.h"

namespace {

using nonode_tu::TconvBwdArgs;
using nonode_tu::tb_groups;

// LDS per group: sX [2 MM - 1][16][ROWP] (Xr_0, (Xr_m, Xs_m)), sG [2 MM][16][ROWP] ((gYr_m, gYi_m));
// shared sCos / sSin [MM * TMAX]: dynamic (93 KB at 2 modes x 3 groups, 152 KB at 9 modes x 1)
// At <= 2 modes the backward mixing fragments (2 MM x 4096 floats) are staged in LDS once per
// workgroup too: read from L2 they were 32 KB per wave and tile.
constexpr bool tb_wlds(int MM) { return MM <= 2; }
constexpr size_t tconv_bwd_lds_bytes(int MM) {
  return ((size_t)tb_groups(MM) * (4 * MM - 1) * 16 * ROWP + 2 * (size_t)MM * TMAX +
          (tb_wlds(MM) ? (size_t)2 * MM * 4096 : 0)) * sizeof(float);
}
// TB: compile-time frame bound (10 for T <= 10, else TMAX), in chunks of TC frames: each chunk's loads
// (h, the output gradient and its LeakyReLU mask words) are issued together, unconditionally with the
// frame index clamped to T - 1, before any of them is used. (Round 5's loads sat under `if (t < T)`
// inside a TMAX-frame loop: every frame became a branch, a single load and a wait, i.e. one memory
// latency per frame in steps 3 and 4.)
template <int MM, int TB>
__global__ __launch_bounds__(256 * tb_groups(MM)) void tconv_bwd_kernel(TconvBwdArgs p) {
  constexpr int TC = TB % 5 == 0 ? 5 : 4;
  static_assert(TB % TC == 0, "whole frame chunks");
  constexpr int NG = tb_groups(MM);
  static_assert(NG == 1 || 4096 <= (size_t)NG * (4 * MM - 1) * 16 * ROWP, "accumulator hand-off space");
  extern __shared__ __attribute__((aligned(16))) float tb_smem[];
  typedef float Row[16][ROWP];
  const int tid = threadIdx.x, lane = tid & 63, grp = tid >> 8, wave = (tid >> 6) & 3, e = lane & 15, g = lane >> 4;
  Row* sX = reinterpret_cast<Row*>(tb_smem) + grp * (4 * MM - 1);
  Row* sG = sX + (2 * MM - 1);
  float* sCos = reinterpret_cast<float*>(reinterpret_cast<Row*>(tb_smem) + NG * (4 * MM - 1));
  float* sSin = sCos + MM * TMAX;
  float* sWb = sSin + MM * TMAX;   // tb_wlds(MM): the backward mixing fragments
  const int T = p.T, BN = p.BN;
  if constexpr (tb_wlds(MM)) {
    for (int i = tid; i < 2 * MM * 1024; i += 256 * NG)
      reinterpret_cast<f4*>(sWb)[i] = reinterpret_cast<const f4*>(p.wb)[i];
  }
  const float* wb = tb_wlds(MM) ? sWb : p.wb;
  if (tid < MM * T) {
    const int m = tid / T, t = tid - (tid / T) * T;
    const double ang = 2.0 * (double)m * (double)t / (double)T;
    sCos[m * TMAX + t] = (float)cospi(ang);
    sSin[m * TMAX + t] = (float)sinpi(ang);
  }
  const int ch = 16 * wave + 4 * g;   // this lane's 4 channels (input side and output side)
  f4 aR[MM][4], aI[MM][4];            // gWr_m / gWi_m rows 16 wave.., column tiles it
#pragma unroll
  for (int m = 0; m < MM; ++m)
#pragma unroll
    for (int it = 0; it < 4; ++it) aR[m][it] = aI[m][it] = f4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  // every group runs the same number of trips (the barriers are the workgroup's); a group past the
  // last tile works on zeros (tile clamped, nothing stored)
  for (int base = blockIdx.x * NG; base < p.ntiles; base += gridDim.x * NG) {
    const bool gact = base + grp < p.ntiles;
    const int tile = gact ? base + grp : p.ntiles - 1;
    const int col = tile * 16 + e;
    const bool cvalid = gact && col < BN;
    const int c = col < BN ? col : BN - 1;
    auto hval = [&](const float* base, int t) -> f4 {
      return *reinterpret_cast<const f4*>(base + ((size_t)t * BN + c) * 64 + ch);
    };
    // ---- 1: DFT ----
    {
      f4 Xr[MM], Xs[MM];
#pragma unroll
      for (int m = 0; m < MM; ++m) { Xr[m] = f4{0.f, 0.f, 0.f, 0.f}; Xs[m] = Xr[m]; }
#pragma unroll
      for (int t0 = 0; t0 < TB; t0 += TC) {
        f4 hv[TC];
#pragma unroll
        for (int i = 0; i < TC; ++i) hv[i] = hval(p.h, t0 + i < T ? t0 + i : T - 1);
#pragma unroll
        for (int i = 0; i < TC; ++i) {
          const int t = t0 + i;
          if (t < T) {
#pragma unroll
            for (int m = 0; m < MM; ++m) {
              Xr[m] += hv[i] * sCos[m * TMAX + t];
              if (m > 0) Xs[m] += hv[i] * sSin[m * TMAX + t];
            }
          }
        }
      }
      const f4 z = {0.f, 0.f, 0.f, 0.f};
      *reinterpret_cast<f4*>(&sX[0][e][ch]) = cvalid ? Xr[0] : z;
#pragma unroll
      for (int m = 1; m < MM; ++m) {
        *reinterpret_cast<f4*>(&sX[2 * m - 1][e][ch]) = cvalid ? Xr[m] : z;
        *reinterpret_cast<f4*>(&sX[2 * m][e][ch]) = cvalid ? Xs[m] : z;
      }
    }
    __syncthreads();
    auto mix = [&](f4& acc, const float* frags, int mat, const float (*src)[ROWP]) {
      f4 in[4];
      load_ecl(in, &src[e][0], g);
      const float* wf = frags + (size_t)mat * 4096;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const f4 a = *reinterpret_cast<const f4*>(wf + ((wave * 4 + mt) * 64 + lane) * 4);
#pragma unroll
        for (int q = 0; q < 4; ++q) acc = mfma(a[q], in[mt][q], acc);
      }
    };
    // the forward's LeakyReLU decisions for this lane's element (column e, channels ch..ch+3): word
    // ((t * ntiles + tile) * 4 + e / 4) * 4 + q, bit ((e & 3) << 4) | (ch >> 2)
    const unsigned long long* mrow = p.mask + ((size_t)tile * 4 + (e >> 2)) * 4;
    const int mbit = ((e & 3) << 4) | (ch >> 2);
    const size_t mstride = (size_t)p.ntiles * 16;
    // ---- 3: gy and its spectral coefficients ----
    {
      f4 gR[MM], gI[MM];
#pragma unroll
      for (int m = 0; m < MM; ++m) { gR[m] = f4{0.f, 0.f, 0.f, 0.f}; gI[m] = gR[m]; }
#pragma unroll
      for (int t0 = 0; t0 < TB; t0 += TC) {
        f4 gy[TC];
        unsigned long long mw[TC][4];
#pragma unroll
        for (int i = 0; i < TC; ++i) {
          const int tc = t0 + i < T ? t0 + i : T - 1;
          gy[i] = hval(p.gout, tc);
#pragma unroll
          for (int q = 0; q < 4; ++q) mw[i][q] = mrow[tc * mstride + q];
        }
#pragma unroll
        for (int i = 0; i < TC; ++i) {
          const int t = t0 + i;
          if (t < T) {
#pragma unroll
            for (int q = 0; q < 4; ++q) gy[i][q] *= ((mw[i][q] >> mbit) & 1) ? 1.f : 0.01f;
#pragma unroll
            for (int m = 0; m < MM; ++m) {
              gR[m] += gy[i] * sCos[m * TMAX + t];
              gI[m] -= gy[i] * sSin[m * TMAX + t];
            }
          }
        }
      }
#pragma unroll
      for (int m = 0; m < MM; ++m) {
        const float cm = ((m == 0 || 2 * m == T) ? 1.f : 2.f) / (float)T;
        const f4 z = {0.f, 0.f, 0.f, 0.f};
        *reinterpret_cast<f4*>(&sG[2 * m][e][ch]) = cvalid ? gR[m] * cm : z;
        *reinterpret_cast<f4*>(&sG[2 * m + 1][e][ch]) = cvalid ? gI[m] * cm : z;
      }
    }
    __syncthreads();
    // ---- 4: backward mixing (input tile mo = wave) and gh ----
    {
      f4 gXr[MM], gXi[MM];
#pragma unroll
      for (int m = 0; m < MM; ++m) {
        gXr[m] = f4{0.f, 0.f, 0.f, 0.f};
        gXi[m] = f4{0.f, 0.f, 0.f, 0.f};
        mix(gXr[m], wb, 2 * m + 0, sG[2 * m]);       //  Wr gYr
        mix(gXr[m], wb, 2 * m + 1, sG[2 * m + 1]);   //  Wi gYi
        mix(gXi[m], wb, 2 * m + 0, sG[2 * m + 1]);   //  Wr gYi
        f4 t = {0.f, 0.f, 0.f, 0.f};
        mix(t, wb, 2 * m + 1, sG[2 * m]);            //  Wi gYr
        gXi[m] -= t;
      }
      if (cvalid) {
#pragma unroll
        for (int t0 = 0; t0 < TB; t0 += TC) {
          f4 o[TC];
#pragma unroll
          for (int i = 0; i < TC; ++i) o[i] = hval(p.gout, t0 + i < T ? t0 + i : T - 1);
#pragma unroll
          for (int i = 0; i < TC; ++i) {
            const int t = t0 + i;
            if (t < T) {
#pragma unroll
              for (int m = 0; m < MM; ++m) o[i] += gXr[m] * sCos[m * TMAX + t] - gXi[m] * sSin[m * TMAX + t];
              *reinterpret_cast<f4*>(p.gh + ((size_t)t * BN + c) * 64 + ch) = o[i];
            }
          }
        }
      }
    }
    // ---- 5: weight gradient over this tile's 16 columns ----
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int row = 4 * g + ks;
#pragma unroll
      for (int m = 0; m < MM; ++m) {
        const float xr = sX[m == 0 ? 0 : 2 * m - 1][row][16 * wave + e];
        const float xs = m == 0 ? 0.f : sX[2 * m][row][16 * wave + e];
#pragma unroll
        for (int it = 0; it < 4; ++it) {
          const float gyr = sG[2 * m][row][16 * it + e], gyi = sG[2 * m + 1][row][16 * it + e];
          aR[m][it] = mfma(xr, gyr, aR[m][it]);          // Xr gYr
          aI[m][it] = mfma(xr, gyi, aI[m][it]);          // Xr gYi
          if (m > 0) {
            aR[m][it] = mfma(-xs, gyi, aR[m][it]);       // + Xi gYi  (Xi = -Xs)
            aI[m][it] = mfma(xs, gyr, aI[m][it]);        // - Xi gYr
          }
        }
      }
    }
    __syncthreads();
  }
  // groups 1 .. NG-1 hand their accumulators to group 0 through LDS (the sX / sG space), one group and
  // one [m][re|im] block (4096 floats) at a time, in order
  float* sAcc = tb_smem;
  const int al = (wave * 64 + lane) * 4;   // this lane's f4 slot within one [it] block of 1024
#pragma unroll 1
  for (int gsrc = 1; gsrc < NG; ++gsrc) {
#pragma unroll
    for (int m = 0; m < MM; ++m)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        f4 (&a)[4] = c == 0 ? aR[m] : aI[m];
        if (grp == gsrc) {
#pragma unroll
          for (int it = 0; it < 4; ++it) *reinterpret_cast<f4*>(sAcc + it * 1024 + al) = a[it];
        }
        __syncthreads();
        if (grp == 0) {
#pragma unroll
          for (int it = 0; it < 4; ++it) a[it] += *reinterpret_cast<const f4*>(sAcc + it * 1024 + al);
        }
        __syncthreads();
      }
  }
  if (grp != 0) return;
  float* wp = p.wpart + (size_t)blockIdx.x * p.M * 2 * 4096;
#pragma unroll
  for (int m = 0; m < MM; ++m)
#pragma unroll
    for (int it = 0; it < 4; ++it)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = 16 * wave + 4 * g + q, o = 16 * it + e;
        wp[((m * 2 + 0) * 64 + i) * 64 + o] = aR[m][it][q];
        wp[((m * 2 + 1) * 64 + i) * 64 + o] = aI[m][it][q];
      }
}

}  // namespace

namespace nonode_tu {
int launch_tconv_bwd(int M, TconvBwdArgs a, int G, hipStream_t s) {
  auto go = [&](auto mm) {
    constexpr int MM = decltype(mm)::value;
    static std::once_flag once;
    std::call_once(once, [] {
      hipFuncSetAttribute((const void*)tconv_bwd_kernel<MM, 10>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)tconv_bwd_lds_bytes(MM));
      hipFuncSetAttribute((const void*)tconv_bwd_kernel<MM, TMAX>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)tconv_bwd_lds_bytes(MM));
    });
    if (a.T <= 10)
      hipLaunchKernelGGL((tconv_bwd_kernel<MM, 10>), dim3(G), dim3(256 * tb_groups(MM)), tconv_bwd_lds_bytes(MM), s, a);
    else
      hipLaunchKernelGGL((tconv_bwd_kernel<MM, TMAX>), dim3(G), dim3(256 * tb_groups(MM)), tconv_bwd_lds_bytes(MM), s, a);
  };
  switch (M) {
    case 1: go(std::integral_constant<int, 1>{}); break;
    case 2: go(std::integral_constant<int, 2>{}); break;
    case 3: go(std::integral_constant<int, 3>{}); break;
    case 4: go(std::integral_constant<int, 4>{}); break;
    case 5: go(std::integral_constant<int, 5>{}); break;   // num_modes = 5 (model_confs.yaml:12)
    case 6: go(std::integral_constant<int, 6>{}); break;
    case 7: go(std::integral_constant<int, 7>{}); break;
    case 8: go(std::integral_constant<int, 8>{}); break;
    case 9: go(std::integral_constant<int, 9>{}); break;
    default: return fail(NONODE_EUNSUPPORTED, "tconv_bwd: modes=%d", M);
  }
  return check_launch("tconv_bwd_kernel");
}
}  // namespace nonode_tu
