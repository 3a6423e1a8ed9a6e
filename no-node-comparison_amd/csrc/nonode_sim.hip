// N-body simulators on the GPU: the reference's synthetic data generators.
//
//   sim_charged_kernel  ChargedParticlesSim.sample_trajectory (synthetic_sim.py:220-296): Coulomb
//                       forces q_i q_j (x_i - x_j) / |x_i - x_j|^3, per-component clamp +-max_F,
//                       the reference's leapfrog (initial half kick, then drift / sample / kick)
//   sim_gravity_kernel  GravitySim.sample_trajectory_batch (synthetic_sim.py:407-481): softened
//                       gravity a_i = G sum_j m_j (x_j - x_i) (|x_j - x_i|^2 + s^2)^-3/2,
//                       kick-drift-kick, samples (x, v, a m) every sample_freq steps
//
// float64 like the reference's numpy. One thread per particle; a workgroup holds floor(64 / N)
// whole trajectories when N <= 32 (three at N = 20, so 60 of 64 lanes work), else one trajectory
// of ceil(N / 64) waves. The positions of the current step live in LDS. The per-pair arithmetic
// mirrors the reference's expression order (squared distance of ChargedParticlesSim._l2 as
// |a|^2 + |b|^2 - 2 a.b, no FMA contraction); x^(3/2) is x sqrt(x) (within an ulp of numpy's pow).
// Short horizons agree to rounding; the reference's numpy reductions sum in a different order,
// and both trajectories are chaotic over long ones.
//
// Included at the end of nonode.hip (same translation unit).

namespace {

constexpr int SIM_NMAX = 1024;

__device__ __forceinline__ double dmul(double a, double b) { return __dmul_rn(a, b); }
__device__ __forceinline__ double dadd(double a, double b) { return __dadd_rn(a, b); }
__device__ __forceinline__ double dsub(double a, double b) { return __dsub_rn(a, b); }

struct SimChargedArgs {
  int S, per_wg, N, T, freq, T_save;
  double dt, max_F, strength;
  const double* loc0; const double* vel0;   // [S][3][N] (already clamped / normalised)
  const double* q;                          // [S][N]
  double* loc_out; double* vel_out;         // [S][T_save][3][N]
};

// thread -> (trajectory, particle): G trajectories of N particles per workgroup
struct SimSlot {
  int s, i, base;   // trajectory, particle, first LDS slot of the trajectory
  bool act;
};
__device__ __forceinline__ SimSlot sim_slot(int S, int N, int G) {
  SimSlot r;
  const int t = threadIdx.x, ls = t / N;
  r.i = t - ls * N;
  r.s = blockIdx.x * G + ls;
  r.base = ls * N;
  r.act = ls < G && r.s < S;
  return r;
}

__global__ __launch_bounds__(1024) void sim_charged_kernel(SimChargedArgs a) {
  __shared__ double sx[3][SIM_NMAX];
  __shared__ double sq[SIM_NMAX];
  __shared__ double sn[SIM_NMAX];   // |x_j|^2 (ChargedParticlesSim._l2's row norms)
  const int N = a.N;
  const SimSlot sl = sim_slot(a.S, N, a.per_wg);
  const int s = sl.s, i = sl.i, o = sl.base;
  const bool act = sl.act;
  double x[3] = {0.0, 0.0, 0.0}, v[3] = {0.0, 0.0, 0.0}, qi = 0.0;
  if (act) {
    for (int d = 0; d < 3; ++d) {
      x[d] = a.loc0[((size_t)s * 3 + d) * N + i];
      v[d] = a.vel0[((size_t)s * 3 + d) * N + i];
    }
    qi = a.q[(size_t)s * N + i];
    sq[o + i] = qi;
  }
  auto kick = [&]() {
    if (act) {
      sx[0][o + i] = x[0]; sx[1][o + i] = x[1]; sx[2][o + i] = x[2];
      sn[o + i] = dadd(dadd(dmul(x[0], x[0]), dmul(x[1], x[1])), dmul(x[2], x[2]));
    }
    __syncthreads();
    if (act) {
      double F[3] = {0.0, 0.0, 0.0};
      const double ni = sn[o + i];
      // branch-free over j (the self pair adds an exact 0, fill_diagonal(forces_size, 0)), so the
      // compiler can overlap the divide / sqrt chains of consecutive senders; the sums keep the
      // reference's j order
#pragma unroll 4
      for (int j = 0; j < N; ++j) {
        const bool self = j == i;
        const double xj0 = sx[0][o + j], xj1 = sx[1][o + j], xj2 = sx[2][o + j];
        const double dot = dadd(dadd(dmul(x[0], xj0), dmul(x[1], xj1)), dmul(x[2], xj2));
        const double l2 = self ? 1.0 : dsub(dadd(ni, sn[o + j]), dmul(2.0, dot));
        const double fs = self ? 0.0 : dmul(a.strength, qi * sq[o + j]) / dmul(l2, sqrt(l2));
        F[0] = dadd(F[0], dmul(fs, dsub(x[0], xj0)));
        F[1] = dadd(F[1], dmul(fs, dsub(x[1], xj1)));
        F[2] = dadd(F[2], dmul(fs, dsub(x[2], xj2)));
      }
      for (int d = 0; d < 3; ++d) {
        const double f = F[d] > a.max_F ? a.max_F : (F[d] < -a.max_F ? -a.max_F : F[d]);
        v[d] = dadd(v[d], dmul(a.dt, f));
      }
    }
    __syncthreads();
  };
  kick();   // the half step before the loop (synthetic_sim.py:240-262)
  int counter = 0;
  for (int t = 1; t < a.T; ++t) {
    if (act)
      for (int d = 0; d < 3; ++d) x[d] = dadd(x[d], dmul(a.dt, v[d]));
    if (t % a.freq == 0) {
      if (act && counter < a.T_save)
        for (int d = 0; d < 3; ++d) {
          const size_t o = (((size_t)s * a.T_save + counter) * 3 + d) * N + i;
          a.loc_out[o] = x[d];
          a.vel_out[o] = v[d];
        }
      ++counter;
    }
    kick();
  }
}

struct SimGravityArgs {
  int S, per_wg, N, T, freq, T_save;
  double dt, G, soft2;
  const double* pos0; const double* vel0;   // [S][N][3]
  const double* m;                          // [S][N]
  double* pos_out; double* vel_out; double* force_out;   // [S][T_save][N][3]
};

__global__ __launch_bounds__(1024) void sim_gravity_kernel(SimGravityArgs a) {
  __shared__ double sx[3][SIM_NMAX];
  __shared__ double sm[SIM_NMAX];
  const int N = a.N;
  const SimSlot sl = sim_slot(a.S, N, a.per_wg);
  const int s = sl.s, i = sl.i, o = sl.base;
  const bool act = sl.act;
  double x[3] = {0.0, 0.0, 0.0}, v[3] = {0.0, 0.0, 0.0}, acc[3] = {0.0, 0.0, 0.0}, mi = 0.0;
  if (act) {
    for (int d = 0; d < 3; ++d) {
      x[d] = a.pos0[((size_t)s * N + i) * 3 + d];
      v[d] = a.vel0[((size_t)s * N + i) * 3 + d];
    }
    mi = a.m[(size_t)s * N + i];
    sm[o + i] = mi;
  }
  auto accel = [&]() {   // compute_acceleration_batch (synthetic_sim.py:458-481)
    if (act) { sx[0][o + i] = x[0]; sx[1][o + i] = x[1]; sx[2][o + i] = x[2]; }
    __syncthreads();
    if (act) {
      double A[3] = {0.0, 0.0, 0.0};
#pragma unroll 4
      for (int j = 0; j < N; ++j) {
        const double dx = dsub(sx[0][o + j], x[0]), dy = dsub(sx[1][o + j], x[1]), dz = dsub(sx[2][o + j], x[2]);
        const double r2 = dadd(dadd(dadd(dmul(dx, dx), dmul(dy, dy)), dmul(dz, dz)), a.soft2);
        const double inv = r2 > 0.0 ? 1.0 / dmul(r2, sqrt(r2)) : 0.0;
        const double w = sm[o + j];
        A[0] = dadd(A[0], dmul(dmul(dx, inv), w));
        A[1] = dadd(A[1], dmul(dmul(dy, inv), w));
        A[2] = dadd(A[2], dmul(dmul(dz, inv), w));
      }
      for (int d = 0; d < 3; ++d) acc[d] = dmul(a.G, A[d]);
    }
    __syncthreads();
  };
  accel();
  const double hdt = a.dt / 2.0;
  for (int t = 0; t < a.T; ++t) {
    if (t % a.freq == 0 && act) {
      const int k = t / a.freq;
      for (int d = 0; d < 3; ++d) {
        const size_t o = (((size_t)s * a.T_save + k) * N + i) * 3 + d;
        a.pos_out[o] = x[d];
        a.vel_out[o] = v[d];
        a.force_out[o] = dmul(acc[d], mi);
      }
    }
    if (act)
      for (int d = 0; d < 3; ++d) {
        v[d] = dadd(v[d], dmul(acc[d], hdt));   // (1/2) kick
        x[d] = dadd(x[d], dmul(v[d], a.dt));    // drift
      }
    accel();
    if (act)
      for (int d = 0; d < 3; ++d) v[d] = dadd(v[d], dmul(acc[d], hdt));
  }
}

// trajectories per workgroup and threads per workgroup
int sim_group(int N) { return N <= 32 ? 64 / N : 1; }
int sim_block(int N) { return N <= 32 ? 64 : ((N + 63) / 64) * 64; }

}  // namespace

extern "C" {

int nonode_sim_charged(int S, int N, int T, int sample_freq, double dt, double max_F, double strength,
                       const double* loc0, const double* vel0, const double* charges, double* loc_out,
                       double* vel_out, void* stream) {
  if (S <= 0 || N < 2 || N > SIM_NMAX || T <= 0 || sample_freq <= 0 || T % sample_freq)
    return fail(NONODE_EINVAL, "sim_charged: S=%d N=%d T=%d sample_freq=%d", S, N, T, sample_freq);
  if (!loc0 || !vel0 || !charges || !loc_out || !vel_out) return fail(NONODE_EINVAL, "sim_charged: null pointer");
  const int G = sim_group(N);
  SimChargedArgs a{S, G, N, T, sample_freq, T / sample_freq - 1, dt, max_F, strength, loc0, vel0, charges, loc_out,
                   vel_out};
  ProfScope prof(PROF_SIM_CHARGED, (hipStream_t)stream);
  hipLaunchKernelGGL(sim_charged_kernel, dim3((S + G - 1) / G), dim3(sim_block(N)), 0, (hipStream_t)stream, a);
  return check_launch("sim_charged_kernel");
}

int nonode_sim_gravity(int S, int N, int T, int sample_freq, double dt, double G, double softening,
                       const double* pos0, const double* vel0, const double* mass, double* pos_out, double* vel_out,
                       double* force_out, void* stream) {
  if (S <= 0 || N < 1 || N > SIM_NMAX || T <= 0 || sample_freq <= 0 || T % sample_freq)
    return fail(NONODE_EINVAL, "sim_gravity: S=%d N=%d T=%d sample_freq=%d", S, N, T, sample_freq);
  if (!pos0 || !vel0 || !mass || !pos_out || !vel_out || !force_out)
    return fail(NONODE_EINVAL, "sim_gravity: null pointer");
  const int Gs = sim_group(N);
  SimGravityArgs a{S, Gs, N, T, sample_freq, T / sample_freq, dt, G, softening * softening, pos0, vel0, mass,
                   pos_out, vel_out, force_out};
  ProfScope prof(PROF_SIM_GRAVITY, (hipStream_t)stream);
  hipLaunchKernelGGL(sim_gravity_kernel, dim3((S + Gs - 1) / Gs), dim3(sim_block(N)), 0, (hipStream_t)stream, a);
  return check_launch("sim_gravity_kernel");
}

}  // extern "C"
