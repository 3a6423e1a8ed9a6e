// EGNN_Layer with flat=True (EGNO main_simulation_simple_no.py --flat; basic.py:38-40: every BaseMLP
// 4x wide, 256 hidden channels, with Tanh): the forward (inference) on gfx950.
//
// Included at the end of nonode.hip (same translation unit: the ECL helpers, mfma_dense, the
// TimeConv and embedding launches). No BASELINE configuration uses flat=True, so this path is built
// for parity, not for speed: exact f32 MFMAs (v_mfma_f32_16x16x4_f32, mfma_dense) in three launches
// per layer, the 256-wide activations in registers in the ECL layout of 16 k-steps (lane (e, g) of
// column e holds channels 16 i + 4 g + q, i = 0..15, q = 0..3: the B operand of mfma_dense<16> and,
// block by block, the accumulators of four mfma_dense<KT> over 64-row slices).
//   flat_proj_kernel  P = W1[h_i] h + b1, Q = W1[h_j] h   (the edge MLP's first Linear, per node)
//   flat_edge_kernel  per receiver tile, all N-1 sender offsets: m = Tanh(W2 Tanh(P_i + Q_j +
//                     W1[s|e] [s, e]) + b2), c = wc2 . Tanh(Wc1 m + bc1) + bc2, f = r c; sums of m
//                     and f per receiver in registers (basic.py:167-173, aggregate basic.py:6-31)
//   flat_node_kernel  x += (wv2 . Tanh(Wv1 h + bv1) + bv2) v + clamp(mean f, +-100);
//                     h = Wn2 Tanh(Wn1 [h, sum m] + bn1) + bn2   (basic.py:174-185)

namespace {

// flat blob (floats): f32 MFMA A-operand fragments (pack_frag layout) and natural-order vectors
constexpr int FL_WA = 0;                  // W1[:, h_i columns]: 4 row blocks of 64 x (KT = 4)
constexpr int FL_WB = FL_WA + 4 * 4096;   // W1[:, h_j columns]
constexpr int FL_W2 = FL_WB + 4 * 4096;   // W2 [64][256]: KT = 16
constexpr int FL_WC1 = FL_W2 + 16384;     // Wc1 [256][64]: 4 row blocks, KT = 4
constexpr int FL_WV1 = FL_WC1 + 4 * 4096; // node_v W1 [256][64]
constexpr int FL_WN1 = FL_WV1 + 4 * 4096; // node W1 [256][128]: 4 row blocks, KT = 8
constexpr int FL_WN2 = FL_WN1 + 4 * 8192; // node W2 [64][256]: KT = 16
constexpr int FL_VEC = FL_WN2 + 16384;    // 256-wide vectors, FV_* below
enum : int { FV_B1 = 0, FV_WS, FV_WE0, FV_WE1, FV_WE2, FV_WE3, FV_BC1, FV_WC2, FV_BV1, FV_WV2, FV_BN1, FV_COUNT };
constexpr int FL_VEC64 = FL_VEC + FV_COUNT * 256;   // b2 [64], bn2 [64]
constexpr int FL_SCAL = FL_VEC64 + 128;             // [0] bc2, [1] bv2, [2] norm flag
constexpr int FL_FLOATS = FL_SCAL + 64;
constexpr int FL_EDGE_LDS = 2 * 16384;              // W2 and Wc1 fragments staged per workgroup

struct FlatPackArgs {
  const float *w1, *b1, *w2, *b2, *cw1, *cb1, *cw2, *cb2, *vw1, *vb1, *vw2, *vb2, *nw1, *nb1, *nw2, *nb2;
  int ld1, ne, norm;
  float* blob;
};
// one thread per blob float
__global__ void flat_pack_kernel(FlatPackArgs a) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  float* B = a.blob;
  if (d >= FL_FLOATS) return;
  if (d < FL_WB) {   // W1 h_i columns (EGNO order [s, h_i, h_j, e]: columns 1 .. 64)
    const int b = d >> 12;
    pack_frag(B + FL_WA + b * 4096, a.w1 + (size_t)64 * b * a.ld1, a.ld1, 1, 4, d & 4095, 1.f);
  } else if (d < FL_W2) {
    const int dd = d - FL_WB, b = dd >> 12;
    pack_frag(B + FL_WB + b * 4096, a.w1 + (size_t)64 * b * a.ld1, a.ld1, 1 + HID, 4, dd & 4095, 1.f);
  } else if (d < FL_WC1) {
    pack_frag(B + FL_W2, a.w2, 256, 0, 16, d - FL_W2, 1.f);
  } else if (d < FL_WV1) {
    const int dd = d - FL_WC1, b = dd >> 12;
    pack_frag(B + FL_WC1 + b * 4096, a.cw1 + 64 * 64 * b, 64, 0, 4, dd & 4095, 1.f);
  } else if (d < FL_WN1) {
    const int dd = d - FL_WV1, b = dd >> 12;
    pack_frag(B + FL_WV1 + b * 4096, a.vw1 + 64 * 64 * b, 64, 0, 4, dd & 4095, 1.f);
  } else if (d < FL_WN2) {
    const int dd = d - FL_WN1, b = dd >> 13;
    pack_frag(B + FL_WN1 + b * 8192, a.nw1 + 64 * 128 * b, 128, 0, 8, dd & 8191, 1.f);
  } else if (d < FL_VEC) {
    pack_frag(B + FL_WN2, a.nw2, 256, 0, 16, d - FL_WN2, 1.f);
  } else if (d < FL_VEC64) {
    const int v = (d - FL_VEC) >> 8, c = (d - FL_VEC) & 255;
    float val = 0.f;
    switch (v) {
      case FV_B1: val = a.b1[c]; break;
      case FV_WS: val = a.w1[(size_t)c * a.ld1]; break;   // the |r|^2 column
      case FV_WE0: case FV_WE1: case FV_WE2: case FV_WE3:
        val = (v - FV_WE0) < a.ne ? a.w1[(size_t)c * a.ld1 + 2 * HID + 1 + (v - FV_WE0)] : 0.f;
        break;
      case FV_BC1: val = a.cb1[c]; break;
      case FV_WC2: val = a.cw2[c]; break;
      case FV_BV1: val = a.vb1[c]; break;
      case FV_WV2: val = a.vw2[c]; break;
      case FV_BN1: val = a.nb1[c]; break;
    }
    B[d] = val;
  } else if (d < FL_SCAL) {
    const int c = d - FL_VEC64;
    B[d] = c < 64 ? a.b2[c] : a.nb2[c - 64];
  } else {
    const int i = d - FL_SCAL;
    B[d] = i == 0 ? a.cb2[0] : (i == 1 ? a.vb2[0] : (i == 2 ? (a.norm ? 1.f : 0.f) : 0.f));
  }
}

// lane's 64 values of a 256-wide natural-order vector / row, ECL-16 layout
__device__ __forceinline__ void load_ecl16(f4 (&d)[16], const float* row, int g) {
#pragma unroll
  for (int i = 0; i < 16; ++i) d[i] = *reinterpret_cast<const f4*>(row + 16 * i + 4 * g);
}
__device__ __forceinline__ void store_ecl16(float* row, const f4 (&s)[16], int g) {
#pragma unroll
  for (int i = 0; i < 16; ++i) *reinterpret_cast<f4*>(row + 16 * i + 4 * g) = s[i];
}
__device__ __forceinline__ void tanh16(f4 (&a)[16]) {
#pragma unroll
  for (int i = 0; i < 16; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) a[i][q] = tanhf(a[i][q]);
}
// out (256 channels) += W x for a 256 x (16 KT) matrix stored as 4 row blocks of mfma_dense<KT> fragments
template <int KT>
__device__ __forceinline__ void mm256(f4 (&out)[16], const float* wf, const f4* in, int lane) {
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    f4 acc[4] = {out[4 * b], out[4 * b + 1], out[4 * b + 2], out[4 * b + 3]};
    mfma_dense<KT>(acc, wf + b * 64 * 16 * KT, in, lane);
#pragma unroll
    for (int mo = 0; mo < 4; ++mo) out[4 * b + mo] = acc[mo];
  }
}
// sum over the 256 channels of w . a (w natural order): the lane's 64 products, then the 4 lane groups
__device__ __forceinline__ float dot256(const f4 (&a)[16], const float* w, int g) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const f4 wv = *reinterpret_cast<const f4*>(w + 16 * i + 4 * g);
#pragma unroll
    for (int q = 0; q < 4; ++q) s = fmaf(wv[q], a[i][q], s);
  }
  return group_sum(s);
}

struct FlatArgs {
  int n_total, n_graphs, N, ne, ef_mod;
  const float* h; const float* x; const float* v; const float* ef; const float* blob;
  float* P; float* Q; float* M; float* F;   // workspace [n][256], [n][256], [n][64], [n][4]
  float* h_out; float* x_out;
};

// P, Q rows of 16 nodes per wave
__global__ __launch_bounds__(256) void flat_proj_kernel(FlatArgs p) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, e = lane & 15, g = lane >> 4;
  const int r0 = (blockIdx.x * 4 + wave) * 16;
  if (r0 >= p.n_total) return;
  const int r = min(r0 + e, p.n_total - 1);
  f4 hin[4];
  load_ecl(hin, p.h + (size_t)r * HID, g);
  f4 acc[16];
  load_ecl16(acc, p.blob + FL_VEC + FV_B1 * 256, g);
  mm256<4>(acc, p.blob + FL_WA, hin, lane);
  if (r0 + e < p.n_total) store_ecl16(p.P + (size_t)r * 256, acc, g);
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = f4{0.f, 0.f, 0.f, 0.f};
  mm256<4>(acc, p.blob + FL_WB, hin, lane);
  if (r0 + e < p.n_total) store_ecl16(p.Q + (size_t)r * 256, acc, g);
}

// one wave per 16-receiver tile, every sender offset k = 1 .. N-1 in turn (receiver r meets sender
// (n + k) mod N of its graph); W2 / Wc1 fragments staged in LDS once per workgroup
__global__ __launch_bounds__(256) void flat_edge_kernel(FlatArgs p) {
  extern __shared__ __attribute__((aligned(16))) float fsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, e = lane & 15, g = lane >> 4;
  for (int i = tid; i < FL_EDGE_LDS / 4; i += 256)
    reinterpret_cast<f4*>(fsm)[i] = reinterpret_cast<const f4*>(p.blob + FL_W2)[i];   // W2 | Wc1 adjacent
  __syncthreads();
  const float* sW2 = fsm;
  const float* sWc1 = fsm + 16384;
  const float* vec = p.blob + FL_VEC;
  const float bc2 = p.blob[FL_SCAL + 0];
  const bool norm = p.blob[FL_SCAL + 2] != 0.f;
  const int N = p.N, Nm1 = N - 1;
  const int r0 = (blockIdx.x * 4 + wave) * 16;
  if (r0 >= p.n_total) return;
  const bool rvalid = r0 + e < p.n_total;
  const int r = rvalid ? r0 + e : p.n_total - 1;
  const int gr = r / N, n = r - gr * N;
  f4 Pr[16];
  load_ecl16(Pr, p.P + (size_t)r * 256, g);
  const float x0 = p.x[(size_t)r * 3 + 0], x1 = p.x[(size_t)r * 3 + 1], x2 = p.x[(size_t)r * 3 + 2];
  const float* efr = p.ef + ((size_t)(gr % p.ef_mod) * N + n) * Nm1 * p.ne;
  f4 Msum[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) Msum[mt] = f4{0.f, 0.f, 0.f, 0.f};
  float F0 = 0.f, F1 = 0.f, F2 = 0.f;
#pragma unroll 1
  for (int k = 1; k < N; ++k) {
    int j = n + k;
    j = j >= N ? j - N : j;
    const int jj = j < n ? j : j - 1;
    const size_t s = (size_t)gr * N + j;
    const float q0 = x0 - p.x[s * 3 + 0], q1 = x1 - p.x[s * 3 + 1], q2 = x2 - p.x[s * 3 + 2];
    float sr = fmaf(q0, q0, fmaf(q1, q1, q2 * q2));
    if (norm) sr = radial_norm(sr);
    float fe[4] = {0.f, 0.f, 0.f, 0.f};
    for (int f = 0; f < p.ne; ++f) fe[f] = efr[(size_t)jj * p.ne + f];
    // a = Tanh(P_r + Q_s + W1[:, s] s + W1[:, e] e)
    f4 a[16];
    load_ecl16(a, p.Q + s * 256, g);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = 16 * i + 4 * g;
      f4 t = Pr[i] + a[i] + *reinterpret_cast<const f4*>(vec + FV_WS * 256 + c) * sr;
#pragma unroll
      for (int f = 0; f < 4; ++f)
        if (f < p.ne) t += *reinterpret_cast<const f4*>(vec + (FV_WE0 + f) * 256 + c) * fe[f];
      a[i] = t;
    }
    tanh16(a);
    // m = Tanh(W2 a + b2)
    f4 m[4];
    load_ecl(m, p.blob + FL_VEC64, g);
    mfma_dense<16>(m, sW2, a, lane);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int q = 0; q < 4; ++q) m[mt][q] = tanhf(m[mt][q]);
    // c = wc2 . Tanh(Wc1 m + bc1) + bc2
    f4 t[16];
    load_ecl16(t, vec + FV_BC1 * 256, g);
    mm256<4>(t, sWc1, m, lane);
    tanh16(t);
    const float c = dot256(t, vec + FV_WC2 * 256, g) + bc2;
    if (rvalid) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) Msum[mt] += m[mt];
      F0 = fmaf(q0, c, F0);
      F1 = fmaf(q1, c, F1);
      F2 = fmaf(q2, c, F2);
    }
  }
  if (rvalid) {
    store_ecl(p.M + (size_t)r * HID, Msum, g);
    if (g == 0) *reinterpret_cast<f4*>(p.F + (size_t)r * 4) = f4{F0, F1, F2, 0.f};
  }
}

// node update of 16 rows per wave
__global__ __launch_bounds__(256) void flat_node_kernel(FlatArgs p) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, e = lane & 15, g = lane >> 4;
  const int r0 = (blockIdx.x * 4 + wave) * 16;
  if (r0 >= p.n_total) return;
  const bool rvalid = r0 + e < p.n_total;
  const int r = rvalid ? r0 + e : p.n_total - 1;
  const float* vec = p.blob + FL_VEC;
  f4 in8[8];
  load_ecl(*reinterpret_cast<f4(*)[4]>(&in8[0]), p.h + (size_t)r * HID, g);
  load_ecl(*reinterpret_cast<f4(*)[4]>(&in8[4]), p.M + (size_t)r * HID, g);
  // phi = wv2 . Tanh(Wv1 h + bv1) + bv2 ;  x += phi v + clamp(mean f, +-100)
  f4 t[16];
  load_ecl16(t, vec + FV_BV1 * 256, g);
  mm256<4>(t, p.blob + FL_WV1, in8, lane);
  tanh16(t);
  const float phi = dot256(t, vec + FV_WV2 * 256, g) + p.blob[FL_SCAL + 1];
  // h = Wn2 Tanh(Wn1 [h, M] + bn1) + bn2
  load_ecl16(t, vec + FV_BN1 * 256, g);
  mm256<8>(t, p.blob + FL_WN1, in8, lane);
  tanh16(t);
  f4 hn[4];
  load_ecl(hn, p.blob + FL_VEC64 + 64, g);
  mfma_dense<16>(hn, p.blob + FL_WN2, t, lane);
  if (rvalid) {
    store_ecl(p.h_out + (size_t)r * HID, hn, g);
    if (g == 0) {
      const float inv = 1.f / (float)(p.N - 1);
      const f4 Fr = *reinterpret_cast<const f4*>(p.F + (size_t)r * 4);
#pragma unroll
      for (int d = 0; d < 3; ++d)
        p.x_out[(size_t)r * 3 + d] =
            p.x[(size_t)r * 3 + d] + phi * p.v[(size_t)r * 3 + d] + fminf(fmaxf(Fr[d] * inv, -100.f), 100.f);
    }
  }
}

// one flat EGNN layer: three launches (projections, edges, node update); ws = n x 580 floats
int launch_flat_layer(int n_graphs, int N, int ne, int ef_mod, const float* h, const float* x, const float* v,
                      const float* ef, const float* blob, float* h_out, float* x_out, float* ws, hipStream_t s) {
  static std::once_flag once;
  std::call_once(once, [] {
    hipFuncSetAttribute((const void*)flat_edge_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                        FL_EDGE_LDS * 4);
  });
  FlatArgs a;
  a.n_total = n_graphs * N; a.n_graphs = n_graphs; a.N = N; a.ne = ne; a.ef_mod = ef_mod;
  a.h = h; a.x = x; a.v = v; a.ef = ne ? ef : blob; a.blob = blob;
  const size_t n = (size_t)a.n_total;
  a.P = ws; a.Q = ws + n * 256; a.M = ws + n * 512; a.F = ws + n * 576;
  a.h_out = h_out; a.x_out = x_out;
  const int blocks = (int)((n + 63) / 64);
  hipLaunchKernelGGL(flat_proj_kernel, dim3(blocks), dim3(256), 0, s, a);
  if (int rc = check_launch("flat_proj_kernel")) return rc;
  hipLaunchKernelGGL(flat_edge_kernel, dim3(blocks), dim3(256), FL_EDGE_LDS * 4, s, a);
  if (int rc = check_launch("flat_edge_kernel")) return rc;
  hipLaunchKernelGGL(flat_node_kernel, dim3(blocks), dim3(256), 0, s, a);
  return check_launch("flat_node_kernel");
}

// ---- the reverse pass of one flat layer (EGNO(flat=True) training; basic.py:38-40, 107-186 reversed) ----
// Parity-first like the forward (exact f32 MFMAs): the per-node and per-edge reverse of the 256-wide
// Tanh MLPs runs in two kernels; the weight gradients are plain GEMMs over the nodes / edges of the
// operands these kernels write (dW = G^T A, summed by the host with a BLAS GEMM).
// Transposed fragments (flat backward blob): 64 x 256 matrices as 16 k-steps of mfma_dense<16>, 256 x 64
// matrices as 4 row blocks of mfma_dense<4>.
constexpr int FB_WV1T = 0;                   // WV1^T  [64][256]
constexpr int FB_WN1HT = FB_WV1T + 16384;    // WN1[:, :64]^T [64][256]
constexpr int FB_WN1MT = FB_WN1HT + 16384;   // WN1[:, 64:]^T [64][256]
constexpr int FB_WC1T = FB_WN1MT + 16384;    // Wc1^T  [64][256]
constexpr int FB_W2T = FB_WC1T + 16384;      // W2^T   [256][64]: 4 row blocks
constexpr int FB_WN2T = FB_W2T + 16384;      // WN2^T  [256][64]: 4 row blocks
constexpr int FB_FLOATS = FB_WN2T + 16384;
// per-node / per-edge operand rows of the reverse pass (floats)
constexpr int FN_GHP = 0, FN_GM = 64, FN_GF = 128, FN_GX = 132, FN_GA = 136, FN_GB = 392, FN_T = 648, FN_GT = 904,
              FN_U = 1160, FN_GU = 1416, FN_GPHI = 1672, FN_STRIDE = 1676;
constexpr int FE_A = 0, FE_M = 256, FE_C1 = 320, FE_GZ3 = 576, FE_GZ2 = 832, FE_GPRE = 896, FE_GC = 1152,
              FE_S = 1153, FE_FE = 1154, FE_STRIDE = 1160;   // FE_S: the radial input as used; FE_FE: e (4)

// fragment of a transposed source: value (row o, column i) = W[(col_off + i) ld + row_off + o]
__device__ __forceinline__ void pack_frag_tt(float* dst, const float* W, int ld, int row_off, int KT, int d) {
  const int q = d & 3, l = (d >> 2) & 63, rest = d >> 8;
  const int mt = rest % KT, mo = rest / KT;
  const int o = 16 * mo + (l & 15), i = 16 * mt + 4 * (l >> 4) + q;
  dst[d] = W[(size_t)i * ld + row_off + o];
}
__global__ void flat_pack_bwd_kernel(FlatPackArgs a, float* bb) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= FB_FLOATS) return;
  const int sec = d >> 14, dd = d & 16383;
  switch (sec) {
    case 0: pack_frag_tt(bb + FB_WV1T, a.vw1, 64, 0, 16, dd); break;
    case 1: pack_frag_tt(bb + FB_WN1HT, a.nw1, 128, 0, 16, dd); break;
    case 2: pack_frag_tt(bb + FB_WN1MT, a.nw1, 128, 64, 16, dd); break;
    case 3: pack_frag_tt(bb + FB_WC1T, a.cw1, 64, 0, 16, dd); break;
    case 4: pack_frag_tt(bb + FB_W2T + (dd >> 12) * 4096, a.w2, 256, 64 * (dd >> 12), 4, dd & 4095); break;
    case 5: pack_frag_tt(bb + FB_WN2T + (dd >> 12) * 4096, a.nw2, 256, 64 * (dd >> 12), 4, dd & 4095); break;
  }
}

struct FlatBwdArgs {
  int n_total, N, ne, ef_mod;
  const float* h; const float* x; const float* v; const float* ef; const float* blob; const float* bb;
  const float* P; const float* Q; const float* M; const float* F;   // the forward's workspace rows
  const float* gx; const float* gv; const float* gh;                // gradients of the layer's outputs
  float* nops;   // [n][FN_STRIDE]
  float* eops;   // [n (N - 1)][FE_STRIDE], edge (r, k) at r (N - 1) + k - 1
  float* gv_in;  // [n][3]
};
__device__ __forceinline__ void dtanh16(f4 (&g)[16], const f4 (&t)[16]) {   // g *= 1 - t^2
#pragma unroll
  for (int i = 0; i < 16; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) g[i][q] *= 1.f - t[i][q] * t[i][q];
}

// node reverse (basic.py:174-185), 16 rows per wave: gF, gM, the h part that does not go through the
// edges, dL/dv, and the operands of the node-level weight gradients
__global__ __launch_bounds__(256) void flat_node_bwd_kernel(FlatBwdArgs p) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, e = lane & 15;
  const int r0 = (blockIdx.x * 4 + wave) * 16;
  if (r0 >= p.n_total) return;
  const bool rvalid = r0 + e < p.n_total;
  const int r = rvalid ? r0 + e : p.n_total - 1;
  const float* vec = p.blob + FL_VEC;
  float* no = p.nops + (size_t)r * FN_STRIDE;
  f4 in8[8];
  load_ecl(*reinterpret_cast<f4(*)[4]>(&in8[0]), p.h + (size_t)r * HID, g);
  load_ecl(*reinterpret_cast<f4(*)[4]>(&in8[4]), p.M + (size_t)r * HID, g);
  const float gx0 = p.gx[(size_t)r * 3 + 0], gx1 = p.gx[(size_t)r * 3 + 1], gx2 = p.gx[(size_t)r * 3 + 2];
  const float v0 = p.v[(size_t)r * 3 + 0], v1 = p.v[(size_t)r * 3 + 1], v2 = p.v[(size_t)r * 3 + 2];
  // node_v: t = Tanh(WV1 h + bv1), phi = wv2 . t + bv2; x_out = x + phi v + clamp(F / (N - 1))
  f4 t[16];
  load_ecl16(t, vec + FV_BV1 * 256, g);
  mm256<4>(t, p.blob + FL_WV1, in8, lane);
  tanh16(t);
  const float phi = dot256(t, vec + FV_WV2 * 256, g) + p.blob[FL_SCAL + 1];
  const float gphi = gx0 * v0 + gx1 * v1 + gx2 * v2;
  if (rvalid) store_ecl16(no + FN_T, t, g);
  f4 gt[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) gt[i] = *reinterpret_cast<const f4*>(vec + FV_WV2 * 256 + 16 * i + 4 * g) * gphi;
  dtanh16(gt, t);
  if (rvalid) store_ecl16(no + FN_GT, gt, g);
  f4 ghp[4] = {};
  mfma_dense<16>(ghp, p.bb + FB_WV1T, gt, lane);   // WV1^T gt
  // node MLP: u = Tanh(WN1 [h, M] + bn1), h_out = WN2 u + bn2
  f4 u[16];
  load_ecl16(u, vec + FV_BN1 * 256, g);
  mm256<8>(u, p.blob + FL_WN1, in8, lane);
  tanh16(u);
  if (rvalid) store_ecl16(no + FN_U, u, g);
  f4 gho[4];
  load_ecl(gho, p.gh + (size_t)r * HID, g);
  f4 gu[16] = {};
  mm256<4>(gu, p.bb + FB_WN2T, gho, lane);           // WN2^T gh_out
  dtanh16(gu, u);
  if (rvalid) store_ecl16(no + FN_GU, gu, g);
  mfma_dense<16>(ghp, p.bb + FB_WN1HT, gu, lane);    // + WN1[:, :64]^T gu
  f4 gm[4] = {};
  mfma_dense<16>(gm, p.bb + FB_WN1MT, gu, lane);     // WN1[:, 64:]^T gu
  if (rvalid) {
    store_ecl(no + FN_GHP, ghp, g);
    store_ecl(no + FN_GM, gm, g);
    const float inv = 1.f / (float)(p.N - 1);
    const f4 Fr = *reinterpret_cast<const f4*>(p.F + (size_t)r * 4);
    if (g == 0) {
      // clamp(F / (N - 1), +-100) passes the gradient inside the range (torch.clamp: bounds included)
      f4 gF;
      gF[0] = fabsf(Fr[0] * inv) <= 100.f ? gx0 * inv : 0.f;
      gF[1] = fabsf(Fr[1] * inv) <= 100.f ? gx1 * inv : 0.f;
      gF[2] = fabsf(Fr[2] * inv) <= 100.f ? gx2 * inv : 0.f;
      gF[3] = 0.f;
      *reinterpret_cast<f4*>(no + FN_GF) = gF;
      *reinterpret_cast<f4*>(no + FN_GX) = f4{gx0, gx1, gx2, 0.f};   // the edges add their terms here
      no[FN_GPHI] = gphi;
      p.gv_in[(size_t)r * 3 + 0] = p.gv[(size_t)r * 3 + 0] + phi * gx0;
      p.gv_in[(size_t)r * 3 + 1] = p.gv[(size_t)r * 3 + 1] + phi * gx1;
      p.gv_in[(size_t)r * 3 + 2] = p.gv[(size_t)r * 3 + 2] + phi * gx2;
    }
  }
}

// edge reverse (basic.py:107-173), one wave per 16-receiver tile walking the N - 1 sender offsets as the
// forward does: the receiver sums GA (registers) and dL/dx (receiver side), the sender sums GB and
// dL/dx (sender side) by float atomics, and every edge's operands for the edge-level weight gradients
__global__ __launch_bounds__(256) void flat_edge_bwd_kernel(FlatBwdArgs p) {
  extern __shared__ __attribute__((aligned(16))) float fsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, e = lane & 15, g = lane >> 4;
  for (int i = tid; i < FL_EDGE_LDS / 4; i += 256)
    reinterpret_cast<f4*>(fsm)[i] = reinterpret_cast<const f4*>(p.blob + FL_W2)[i];   // W2 | Wc1
  __syncthreads();
  const float* sW2 = fsm;
  const float* sWc1 = fsm + 16384;
  const float* vec = p.blob + FL_VEC;
  const float bc2 = p.blob[FL_SCAL + 0];
  const bool norm = p.blob[FL_SCAL + 2] != 0.f;
  const int N = p.N, Nm1 = N - 1;
  const int r0 = (blockIdx.x * 4 + wave) * 16;
  if (r0 >= p.n_total) return;
  const bool rvalid = r0 + e < p.n_total;
  const int r = rvalid ? r0 + e : p.n_total - 1;
  const int gr = r / N, n = r - gr * N;
  float* nor = p.nops + (size_t)r * FN_STRIDE;
  const float x0 = p.x[(size_t)r * 3 + 0], x1 = p.x[(size_t)r * 3 + 1], x2 = p.x[(size_t)r * 3 + 2];
  const f4 gF = *reinterpret_cast<const f4*>(nor + FN_GF);
  f4 gMr[4];
  load_ecl(gMr, nor + FN_GM, g);
  const float* efr = p.ef + ((size_t)(gr % p.ef_mod) * N + n) * Nm1 * p.ne;
  f4 GA[16] = {};
  float gxr0 = 0.f, gxr1 = 0.f, gxr2 = 0.f;
#pragma unroll 1
  for (int k = 1; k < N; ++k) {
    int j = n + k;
    j = j >= N ? j - N : j;
    const int jj = j < n ? j : j - 1;
    const size_t s = (size_t)gr * N + j;
    float* eo = p.eops + ((size_t)r * Nm1 + (k - 1)) * FE_STRIDE;
    const float q0 = x0 - p.x[s * 3 + 0], q1 = x1 - p.x[s * 3 + 1], q2 = x2 - p.x[s * 3 + 2];
    const float s2 = fmaf(q0, q0, fmaf(q1, q1, q2 * q2));
    const float sr = norm ? radial_norm(s2) : s2;
    float fe[4] = {0.f, 0.f, 0.f, 0.f};
    for (int f = 0; f < p.ne; ++f) fe[f] = efr[(size_t)jj * p.ne + f];
    // forward recompute: a = Tanh(P_r + Q_s + W1[:, s] s + W1[:, e] e), m, c1, c
    f4 a[16];
    load_ecl16(a, p.Q + s * 256, g);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = 16 * i + 4 * g;
      f4 tt = *reinterpret_cast<const f4*>(p.P + (size_t)r * 256 + c) + a[i] +
              *reinterpret_cast<const f4*>(vec + FV_WS * 256 + c) * sr;
#pragma unroll
      for (int f = 0; f < 4; ++f)
        if (f < p.ne) tt += *reinterpret_cast<const f4*>(vec + (FV_WE0 + f) * 256 + c) * fe[f];
      a[i] = tt;
    }
    tanh16(a);
    f4 m[4];
    load_ecl(m, p.blob + FL_VEC64, g);
    mfma_dense<16>(m, sW2, a, lane);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int q = 0; q < 4; ++q) m[mt][q] = tanhf(m[mt][q]);
    f4 c1[16];
    load_ecl16(c1, vec + FV_BC1 * 256, g);
    mm256<4>(c1, sWc1, m, lane);
    tanh16(c1);
    const float c = dot256(c1, vec + FV_WC2 * 256, g) + bc2;
    // reverse: f = r c (gF_r is the gradient of every edge of receiver r: EGNO clamps the mean)
    const float gc = rvalid ? gF[0] * q0 + gF[1] * q1 + gF[2] * q2 : 0.f;
    if (rvalid) {
      store_ecl16(eo + FE_A, a, g);
      store_ecl(eo + FE_M, m, g);
      store_ecl16(eo + FE_C1, c1, g);
      if (g == 0) {
        eo[FE_GC] = gc;
        eo[FE_S] = sr;
#pragma unroll
        for (int f = 0; f < 4; ++f) eo[FE_FE + f] = fe[f];
      }
    }
    // gz3 = gc wc2 (1 - c1^2) (in c1's registers); gm = Wc1^T gz3 + gM_r; gz2 = gm (1 - m^2)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const f4 w = *reinterpret_cast<const f4*>(vec + FV_WC2 * 256 + 16 * i + 4 * g);
#pragma unroll
      for (int q = 0; q < 4; ++q) c1[i][q] = gc * w[q] * (1.f - c1[i][q] * c1[i][q]);
    }
    if (rvalid) store_ecl16(eo + FE_GZ3, c1, g);
    f4 gz2[4] = {gMr[0], gMr[1], gMr[2], gMr[3]};
    if (!rvalid) zero4(gz2);
    mfma_dense<16>(gz2, p.bb + FB_WC1T, c1, lane);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int q = 0; q < 4; ++q) gz2[mt][q] *= 1.f - m[mt][q] * m[mt][q];
    if (rvalid) store_ecl(eo + FE_GZ2, gz2, g);
    // gpre = W2^T gz2 (1 - a^2)
    f4 gp[16] = {};
    mm256<4>(gp, p.bb + FB_W2T, gz2, lane);
    dtanh16(gp, a);
    if (rvalid) store_ecl16(eo + FE_GPRE, gp, g);
    float gs = dot256(gp, vec + FV_WS * 256, g);
    if (norm) gs = s2 < 1e-12f ? gs * 1e12f : 0.f;   // d normalize(s) / ds
    const float gr0 = fmaf(2.f * gs, q0, gF[0] * c), gr1 = fmaf(2.f * gs, q1, gF[1] * c),
                gr2 = fmaf(2.f * gs, q2, gF[2] * c);
    if (rvalid) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        GA[i] += gp[i];
#pragma unroll
        for (int q = 0; q < 4; ++q) atomicAdd(p.nops + s * FN_STRIDE + FN_GB + 16 * i + 4 * g + q, gp[i][q]);
      }
      gxr0 += gr0; gxr1 += gr1; gxr2 += gr2;
      if (g == 0) {
        atomicAdd(p.nops + s * FN_STRIDE + FN_GX + 0, -gr0);
        atomicAdd(p.nops + s * FN_STRIDE + FN_GX + 1, -gr1);
        atomicAdd(p.nops + s * FN_STRIDE + FN_GX + 2, -gr2);
      }
    }
  }
  if (rvalid) {
    store_ecl16(nor + FN_GA, GA, g);
    if (g == 0) {
      atomicAdd(nor + FN_GX + 0, gxr0);
      atomicAdd(nor + FN_GX + 1, gxr1);
      atomicAdd(nor + FN_GX + 2, gxr2);
    }
  }
}

}  // namespace

extern "C" {

size_t nonode_flat_blob_floats(void) { return FL_FLOATS; }

int nonode_pack_layer_flat(const nonode_layer_weights* w, int variant, int hidden, int n_edge_feat, float* blob,
                           void* stream) {
  if (!w || !blob) return fail(NONODE_EINVAL, "pack_layer_flat: null pointer");
  const int flags = variant & ~0xff;
  if ((variant & 0xff) != NONODE_VARIANT_EGNO || (flags & ~NONODE_LAYER_NORM_RADIAL))
    return fail(NONODE_EINVAL, "pack_layer_flat: EGNO layers only (option bits 0x%x)", flags);
  if (hidden != HID || n_edge_feat < 0 || n_edge_feat > 4)
    return fail(NONODE_EUNSUPPORTED, "pack_layer_flat: hidden=%d n_edge_feat=%d", hidden, n_edge_feat);
  if (!w->edge_w1 || !w->edge_b1 || !w->edge_w2 || !w->edge_b2 || !w->coord_w1 || !w->coord_b1 || !w->coord_w2 ||
      !w->coord_b2 || !w->vel_w1 || !w->vel_b1 || !w->vel_w2 || !w->vel_b2 || !w->node_w1 || !w->node_b1 ||
      !w->node_w2 || !w->node_b2)
    return fail(NONODE_EINVAL, "pack_layer_flat: missing weight pointer");
  FlatPackArgs a{w->edge_w1, w->edge_b1, w->edge_w2, w->edge_b2, w->coord_w1, w->coord_b1, w->coord_w2, w->coord_b2,
                 w->vel_w1, w->vel_b1, w->vel_w2, w->vel_b2, w->node_w1, w->node_b1, w->node_w2, w->node_b2,
                 2 * HID + 1 + n_edge_feat, n_edge_feat, (flags & NONODE_LAYER_NORM_RADIAL) ? 1 : 0, blob};
  hipLaunchKernelGGL(flat_pack_kernel, dim3((FL_FLOATS + 255) / 256), dim3(256), 0, (hipStream_t)stream, a);
  return check_launch("flat_pack_kernel");
}

size_t nonode_flat_bwd_blob_floats(void) { return FB_FLOATS; }

int nonode_pack_layer_flat_bwd(const nonode_layer_weights* w, int n_edge_feat, float* bblob, void* stream) {
  if (!w || !bblob || !w->edge_w2 || !w->coord_w1 || !w->vel_w1 || !w->node_w1 || !w->node_w2)
    return fail(NONODE_EINVAL, "pack_layer_flat_bwd: null pointer");
  FlatPackArgs a{w->edge_w1, w->edge_b1, w->edge_w2, w->edge_b2, w->coord_w1, w->coord_b1, w->coord_w2, w->coord_b2,
                 w->vel_w1, w->vel_b1, w->vel_w2, w->vel_b2, w->node_w1, w->node_b1, w->node_w2, w->node_b2,
                 2 * HID + 1 + n_edge_feat, n_edge_feat, 0, nullptr};
  hipLaunchKernelGGL(flat_pack_bwd_kernel, dim3((FB_FLOATS + 255) / 256), dim3(256), 0, (hipStream_t)stream, a, bblob);
  return check_launch("flat_pack_bwd_kernel");
}

size_t nonode_egnn_layer_flat_state_floats(int n_graphs, int N) { return (size_t)n_graphs * N * 580; }

int nonode_egnn_layer_flat(int n_graphs, int N, int n_edge_feat, int ef_mod, const float* h, const float* x,
                           const float* v, const float* edge_fea, const float* blob, float* h_out, float* x_out,
                           float* state, void* stream) {
  if (n_graphs <= 0 || N < 2 || ef_mod <= 0 || n_edge_feat < 0 || n_edge_feat > 4)
    return fail(NONODE_EUNSUPPORTED, "egnn_layer_flat: n_graphs=%d N=%d ef_mod=%d ne=%d", n_graphs, N, ef_mod,
                n_edge_feat);
  if (!h || !x || !v || !blob || !h_out || !x_out || !state || (n_edge_feat > 0 && !edge_fea))
    return fail(NONODE_EINVAL, "egnn_layer_flat: null pointer");
  return launch_flat_layer(n_graphs, N, n_edge_feat, ef_mod, h, x, v, edge_fea, blob, h_out, x_out, state,
                           (hipStream_t)stream);
}

size_t nonode_egnn_layer_flat_bwd_node_floats(int n_graphs, int N) { return (size_t)n_graphs * N * FN_STRIDE; }
size_t nonode_egnn_layer_flat_bwd_edge_floats(int n_graphs, int N) {
  return (size_t)n_graphs * N * (N - 1) * FE_STRIDE;
}

int nonode_egnn_layer_flat_bwd(int n_graphs, int N, int n_edge_feat, int ef_mod, const float* h, const float* x,
                               const float* v, const float* edge_fea, const float* blob, const float* bblob,
                               const float* state, const float* g_x, const float* g_v, const float* g_h,
                               float* node_ops, float* edge_ops, float* g_v_in, void* stream) {
  if (n_graphs <= 0 || N < 2 || ef_mod <= 0 || n_edge_feat < 0 || n_edge_feat > 4)
    return fail(NONODE_EUNSUPPORTED, "egnn_layer_flat_bwd: n_graphs=%d N=%d ef_mod=%d ne=%d", n_graphs, N, ef_mod,
                n_edge_feat);
  if (!h || !x || !v || !blob || !bblob || !state || !g_x || !g_v || !g_h || !node_ops || !edge_ops || !g_v_in ||
      (n_edge_feat > 0 && !edge_fea))
    return fail(NONODE_EINVAL, "egnn_layer_flat_bwd: null pointer");
  static std::once_flag once;
  std::call_once(once, [] {
    hipFuncSetAttribute((const void*)flat_edge_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, FL_EDGE_LDS * 4);
  });
  hipStream_t s = (hipStream_t)stream;
  const size_t n = (size_t)n_graphs * N;
  FlatBwdArgs a;
  a.n_total = (int)n; a.N = N; a.ne = n_edge_feat; a.ef_mod = ef_mod;
  a.h = h; a.x = x; a.v = v; a.ef = n_edge_feat ? edge_fea : blob; a.blob = blob; a.bb = bblob;
  a.P = state; a.Q = state + n * 256; a.M = state + n * 512; a.F = state + n * 576;
  a.gx = g_x; a.gv = g_v; a.gh = g_h;
  a.nops = node_ops; a.eops = edge_ops; a.gv_in = g_v_in;
  // GB and the sender side of dL/dx are float-atomic sums: zeroed first (the whole node rows)
  if (hipMemsetAsync(node_ops, 0, n * FN_STRIDE * sizeof(float), s) != hipSuccess)
    return fail(NONODE_ELAUNCH, "egnn_layer_flat_bwd: memset");
  const int blocks = (int)((n + 63) / 64);
  hipLaunchKernelGGL(flat_node_bwd_kernel, dim3(blocks), dim3(256), 0, s, a);
  if (int rc = check_launch("flat_node_bwd_kernel")) return rc;
  hipLaunchKernelGGL(flat_edge_bwd_kernel, dim3(blocks), dim3(256), FL_EDGE_LDS * 4, s, a);
  return check_launch("flat_edge_bwd_kernel");
}

}  // extern "C"
