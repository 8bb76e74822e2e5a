// tree_core.h -- the cooperative ("tree") synthesis step, written once for host and device.
//
// W lanes cooperate on one utterance (W = 16 on MI355X: four utterances per wave64).
// Each lane owns ND dynamic sections (23..68: glottis, pharynx/mouth, velum taper) and
// NST static ones (trachea, nose, fossa, sinuses) with their in-currents; the persistent
// state of those sections/currents (pressure, wall motion, flows) lives in the lane's
// registers for the whole utterance.  Lanes exchange neighbour data through a per-utterance
// LDS block.  The per-sample system is solved with an LDL^T in arm order (solve_arms): every
// lane eliminates one segment of the tube in registers and DPP row shifts join the segments.
//
// The step is a sequence of phases.  A phase either runs on every lane (`par`), on the
// utterance's lane 0 (`one`) or on the first k lanes (`lanes`), and phases are separated
// by `sync()`.  Phases only read LDS data written by earlier phases, so the same code runs
//   * on the GPU: one lane per thread, sync() = wave-level memory barrier (tds_tree.hip),
//   * on the CPU: the W lanes of a phase one after another (tests/emu, test-only), which
//     lets the decomposition be checked against the oracle without a GPU.
//
// Reference stages restated here (file:line under src/Backend): Tube::interpolate
// Tube.cpp:438-505; TriangularGlottis::calcGeometry/incTime TriangularGlottis.cpp:154-397;
// TdsModel::prepareTimeStep TdsModel.cpp:718-1010 (noise :1188-1708); calcMatrix
// :1785-2039; solve :2231-2314 (replaced by the tree LDL^T of the same matrix);
// updateVariables :2046-2098; radiated flow :687-705; output stage Synthesizer.cpp:614-627.
#pragma once

#include <cstdint>
#include <type_traits>

#if !defined(__HIPCC__)
#include <cmath>
using std::exp;
using std::fabs;
using std::log10;
using std::isfinite;
using std::pow;
using std::sqrt;
using std::fma;
#endif

#include "afs_model.h"
#include "tree_plan.h"

// Keeps the loads above it from being interleaved with the arithmetic below it (device).
#if defined(__HIP_DEVICE_COMPILE__)
#define AFS_SCHED_BARRIER() __builtin_amdgcn_sched_barrier(0)
// the wave's issue priority (s_setprio: the SIMD's arbiter prefers higher values)
#define AFS_SETPRIO(n) __builtin_amdgcn_s_setprio(n)
// s_waitcnt lgkmcnt(0) (gfx9 encoding: vmcnt and expcnt left at their maximum)
#define AFS_LDS_DRAIN() __builtin_amdgcn_s_waitcnt(0xC07F)
#else
#define AFS_SCHED_BARRIER() ((void)0)
#define AFS_SETPRIO(n) ((void)0)
#define AFS_LDS_DRAIN() ((void)0)
#endif

// AFS_RNG_AHEAD = 2: rng_ahead keeps at least two blocks (60 values) of the rand() stream
// pending, in a 128-entry prefix-sum ring, so that a sample with up to five active dipoles (the
// usual four: the glottis source and a tongue constriction, two each) draws without generating
// on the noise phase's chain; 1: one block ahead in a 64-entry ring (rounds 2-5).
#ifndef AFS_RNG_AHEAD
#define AFS_RNG_AHEAD 2
#endif
// AFS_ARM_SCAN = 1: the arm solver's lane-to-lane reduction and back substitution as prefix
// scans (solve_arms); 0: one DPP step per lane of the longest arm (rounds 2-5)
#ifndef AFS_ARM_SCAN
#define AFS_ARM_SCAN 1
#endif
// AFS_WALK_PRESCALED = 1: the arm walk stores Y / d, F / d, E / d for the back substitution
// (arm_back, which needs AFS_BACK_SCALED) instead of 1 / d, Y, F, E
#ifndef AFS_WALK_PRESCALED
#define AFS_WALK_PRESCALED 1
#endif
// AFS_JUNCTION_ADJ = 1: the junction triangle solved by its adjugate (solve_arms)
#ifndef AFS_JUNCTION_ADJ
#define AFS_JUNCTION_ADJ 1
#endif
// AFS_BACK_SCALED = 1: a lane's back substitution with its x-independent terms scaled ahead (arm_back)
#ifndef AFS_BACK_SCALED
#define AFS_BACK_SCALED 1
#endif

namespace afs {
namespace tree {

constexpr int DYN0 = 23;     // first dynamic section
constexpr int NDYNS = 46;    // sections 23..68
constexpr int NDYP = 48;     // dynamic slots of 16 lanes (3 each); absent slots write the sinks
constexpr int NSTATS = 47;   // sections 0..22, 69..92
constexpr double THR = 0.001;  // MIN_DIPOLE_AMP (TdsModel.cpp:1611)

// ---------------------------------------------------------------------------
// Per-utterance LDS block (doubles).  Regions marked (n) are scratch of the noise phases
// and alias the solver arrays, which are only live from the row phase on.
// ---------------------------------------------------------------------------
enum : int {
  // currents; X_U has two extra slots: U_SINK (idle / absent writes) and U_ZERO (0.0)
  X_U = 0, X_UR = X_U + NC + 2, X_UN = X_UR + NUR,
  X_P4 = X_UN + NUN,                                     // p[22], p[23], p[24], p[25]
  // (the dynamic arrays have NDYP slots: the ones past NDYNS are sinks of absent lane slots;
  // X_D has a sink at NS)
  X_E = X_P4 + 4, X_D = X_E + NDYP,                      // E: dynamic sections (s-23), D: all
  X_L = X_D + NS + 1, X_R1 = X_L + NDYP, X_R0 = X_R1 + NDYP,  // dynamic, s-23
  X_RAD = X_R0 + NDYP,                                   // 1 / radius sqrt(pi / A) of the dynamic sections
  X_SMP = X_RAD + NDYP,                                  // dipole samples (41)
  X_UNION = X_SMP + NDIP,
  //   sink slots of the phases before the rows (n): stores of lanes / slots with nothing to store
  X_ACT = X_UNION, X_NOISE_END = X_ACT + 16,
  //   solver
  //   (pivot / rhs with a sink slot at NC and the dummy pivot at NC+1; edges with EDGE_ZERO
  //   and EDGE_SINK after TREE_NE)
  X_DIAG = X_UNION, X_RHS = X_DIAG + NC + 2, X_OFF = X_RHS + NC + 2,
  X_SOLVE_END = X_OFF + TREE_NE + 2,
  X_AFTER = (X_NOISE_END > X_SOLVE_END ? X_NOISE_END : X_SOLVE_END),
  // frame-rate values written by lane 0 at every frame transition
  X_FRAME = X_AFTER,           // teethL, teethR, velL, velR, gL[6], gR[6]
  // persistent small state
  X_RELX = X_FRAME + 16,       // glottis: cur0, cur1, prev0, prev1
  X_GBF = X_RELX + 4,
  X_TONE = X_GBF + 1,          // glottal tone filter: x1..x4, y1..y4
  X_OUTF = X_TONE + 8,         // output Chebyshev: x1..x8, y1..y8
  X_PREVFLOW = X_OUTF + 16,
  X_NONFIN = X_PREVFLOW + 1,
  X_NDRAW = X_NONFIN + 1,      // rand() calls so far (u64; diagnostics: afs_rng_draws)
  X_RNG = X_NDRAW + 1,         // rand(): value ring (64 u32), prefix-sum ring (128 / 64 u32)
  X_GP = X_RNG + (AFS_RNG_AHEAD >= 2 ? 96 : 64),  // interpolated glottis controls (6), 2 spare
  X_RNG_SINK = X_GP + 6,       //   (spare: the sink of rng_ahead's idle stores, outside the solver arrays)
  X_TGLOT = X_GP + 8,          // transglottal-pressure filter x1..x4, y1..y4 (variable entrance loss)
  X_TVEL = X_TGLOT + 8,        // transvelar coupling filters H1, H2: x1..x4, y1..y4 each
  X_TVP = X_TVEL + 16,         // p[43], p[67] after the last update (transvelar filter inputs)
  X_RRAD = X_TVP + 2,          // mouth radiation R and L (section 64), from the network phase
#if AFS_PAIR
  X_RELX2 = X_RRAD + 2,        // wave pairs: the glottis displacements' second buffer (sample_step_pair)
  X_RNGHP = X_RELX2 + 4,       // wave pairs: the rand() ring head and pending count (two int32)
  X_AGLOT = X_RNGHP + 1,       // wave pairs: the upper glottis section's area of this sample (DYN -> STAT)
  X_TOTAL = X_AGLOT + 1,
#else
  X_TOTAL = X_RRAD + 2,
#endif
  // LDS stride of the utterance blocks: 128 B modulo the 256-B bank row, so that the two
  // utterances of a 32-lane LDS lane group (ds_read_b64: lanes 0-31, 32-63) address the
  // same slot through disjoint banks
  X_STRIDE = X_TOTAL + ((16 - X_TOTAL % 32) + 32) % 32
};
static_assert(X_STRIDE % 32 == 16, "utterance blocks offset by half a bank row");

// Phase ids for Exec::mark (cycle accounting in tools/phase_prof; a no-op otherwise).
enum : int {
  PH_GEOMETRY, PH_NETWORK, PH_NOISE, PH_N_AMP, PH_N_RNG,
  PH_ROWS, PH_FORWARD, PH_BACKWARD, PH_UPDATE, PH_OUTPUT, PH_TARGETS,
  // wave pairs (sample_step_pair): the waits at the four barriers, the DYN wave's rand() blocks, the
  // loop's tail (output window, frame transition and its barrier)
  PH_P1WAIT, PH_P2WAIT, PH_P3WAIT, PH_P4WAIT, PH_RNGP, PH_TAIL,
  PH_S_GLOT, PH_S_TGT,  // (the STAT wave's first phase group: the glottis and static network; the targets)
  PH_D_GEO,             // (the DYN wave's interpolation and glottis)
  PH_P0WAIT,            // (the wait at the barrier inside the first phase group, AFS_PAIR_SPLIT1)
  PH_PLACE_HW, PH_PLACE_T0, PH_PLACE_T1,  // (not timed: the pair kernel's wave placement and loop span)
  PH_COUNT
};

// Solver sink / zero slots (see ArmRec).
constexpr int NODE_SINK = NC, U_SINK = NC, U_ZERO = NC + 1, EDGE_ZERO = TREE_NE, EDGE_SINK = TREE_NE + 1;
constexpr uint32_t RHS_DELTA = (uint32_t)(X_RHS - X_DIAG) * 8u;  // bytes from a pivot to its rhs

template <int W>
struct Shape {
  static constexpr int ND = (NDYNS + W - 1) / W;
  static constexpr int NST = (NSTATS + W - 1) / W;
  static constexpr int NSL = ND + NST;
  static constexpr int NDP = (NDIP + W - 1) / W;
};

// Wave pairs (tree_kernel.h, AFS_PAIR): two waves hold the same four utterances, each half of every
// lane's slots -- ROLE_DYN the dynamic ones (and the radiated flow, the output window), ROLE_STAT the
// static ones and the lane-uniform phases (glottis commit, targets, noise, solver, rand() blocks) --
// so that two waves share each SIMD.  ROLE_ALL: one wave does everything (the default kernel).
enum : int { ROLE_ALL = 0, ROLE_DYN = 1, ROLE_STAT = 2 };
template <int ROLE> AFS_HD constexpr bool role_slot(int j, int nd) {
  return ROLE == ROLE_ALL || ((ROLE == ROLE_DYN) == (j < nd));
}

AFS_HD inline int dyn_section(int W, int j, int gl) {
  int k = j * W + gl;
  return k < NDYNS ? DYN0 + k : -1;
}
AFS_HD inline int static_section(int W, int j, int gl) {
  int k = j * W + gl;
  return k < NSTATS ? (k < 23 ? k : k + 46) : -1;
}

// Arm solver lane registers (solve_arms).
struct ArmCarry {
  double Db, Yb;      // pivot and rhs of the lane's boundary (reduced in place)
  double dA, yA;      // the walk's update of the anchor's pivot and rhs
  double F;           // edge anchor - boundary after the walk
  double inv, x;      // 1 / pivot of the boundary after the arm reduction; its solution
  double Fn, ej;      // F of the next lane; edge boundary - junction node (last lanes)
  double e28, e29;    // fossa lane: edges 84-28, 84-29
  double xJ;          // last lanes: the solution of their junction node (then the anchor's)
  double jd[3], jy[3], je[3], xj[3];  // junction lane: triangle pivots, rhs, edges, solutions
  double sm[4];       // AFS_ARM_SCAN: the lane's segment of the pivot recurrence (2x2), then of the rhs / solution
  int sf, sb, end;    // the arm steps this lane reduces in (forward) / solves in (back), -1: none
  bool neg;           // a pivot this lane met was negative (the system is not positive definite)
};
// Up to four doubles handed between lanes (x.pull).
struct D4 { double v[4]; };


// 1/d for the pivots, areas and surfaces: v_rcp_f64 and one Newton step on the device (within
// 11 ulps of the division, profiles/r02ad_f64_ops.txt).  A second step makes it exactly rounded;
// dropping it measured +2.3 % end to end (profiles/r03s_rcp_rows_ab.txt) with the parity
// figures still 5-6 orders inside the bounds and 0 rand() count differences.
// Plain division in the CPU emulator.
AFS_HD inline double pivot_recip(double d) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double r = __builtin_amdgcn_rcp(d);
  const double e = fma(-d, r, 1.0);
  return fma(r, e, r);
#else
  return 1.0 / d;
#endif
}

// Square root of a positive, finite, normal operand (areas, Q, masses x stiffnesses; the
// inputs of this kernel are >= 1e-3): LLVM's correctly rounded f64 sequence (v_rsq_f64 and
// Goldschmidt/Newton steps) without its range scaling and zero/infinity fix-up, bit-identical
// to sqrt() for x >= 2^-767 (tools/microbench/f64_ops.hip checks 3M inputs).  About 40 of
// sqrt()'s 107 cycles of dependent latency are the parts left out.  Host builds call sqrt.
AFS_HD inline double fast_sqrt(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = 0.5 * y;
  const double r = fma(-h, g, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  double d = fma(-g, g, x);
  g = fma(d, h, g);
  d = fma(-g, g, x);
  return fma(d, h, g);
#else
  return sqrt(x);
#endif
}

// Reciprocal and quotient of positive, normal operands (areas, surfaces, capacitances) without
// the scaling/fixup steps of IEEE division: v_rcp_f64 + one Newton step (pivot_recip: within 11
// ulps of 1 / b), and for the quotient one residual correction (within 1 ulp of a / b for the
// operands here, measured on 3 M inputs by tools/microbench/f64_ops.hip).  Host builds (the CPU
// emulator) divide.
AFS_HD inline double fast_rcp(double d) { return pivot_recip(d); }
AFS_HD inline double fast_div(double a, double b) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double r = pivot_recip(b);
  const double q = a * r;
  return fma(r, fma(-b, q, a), q);
#else
  return a / b;
#endif
}

// The interpolation ratio i / hop of sample i of a hop (0 <= i < hop), from inv_hop = 1 / hop
// (correctly rounded, once per launch): q = i * inv_hop, then one correction by the exact remainder
// i - hop q (an fma): the correctly rounded quotient (Markstein's theorem), so bit for bit the
// division the reference and K5 take (tests/test_hop_ratio.py checks every i < hop for every hop up
// to 8192 and sampled hops up to 65536); one multiply and two fmas instead of the ~10 instructions of
// an IEEE division on the sample's chain.  Host builds divide.
AFS_HD inline double hop_ratio(int i, double dhop, double inv_hop) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double di = (double)i;
  const double q = di * inv_hop;
  return fma(fma(-dhop, q, di), inv_hop, q);
#else
  (void)inv_hop;
  return (double)i / dhop;
#endif
}

// x clamped from below (at_least) or above (at_most) at a positive constant c, as the reference's
// `if (x < c) x = c`.  Device: one v_max_f64 / v_min_f64 (the select form is a compare and two
// 32-bit selects of the constant's halves); equal for every x that is not a NaN (a NaN gives c --
// the inputs here are areas, surfaces and controls, finite).  Host builds compare.
AFS_HD inline double at_least(double x, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_fmax(x, c);
#else
  return x < c ? c : x;
#endif
}
// max(x, 0) as the reference's `if (x < 0) x = 0` / `x < 0 ? 0 : x`: one v_max_f64 on the device.
// Differs only for x = -0 (gives +0: every caller adds it to or multiplies it into a value whose
// result is the same either way) and NaN (gives 0: a NaN flow, displacement or control is in the
// system already).
AFS_HD inline double nonneg(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_fmax(x, 0.0);
#else
  return x < 0.0 ? 0.0 : x;
#endif
}
AFS_HD inline double at_most(double x, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_fmin(x, c);
#else
  return x > c ? c : x;
#endif
}

// Word `kind` of a hop record at `ratio` (tree_plan.h plan_word_eval), branch-free on the
// device: every lane evaluates one square root and one quotient and keeps its kind's value.
// The interpolation is K5's and phase_interpolate's (uncontracted), so the area A is bit-identical.
// The words are NOT bit-identical with K5's dense records: PK_SQRT (sqrt A) is exact (fast_sqrt);
// PK_INVA (1 / A), PK_INVD (1 / sqrt(4 A / pi), here sqrt((4 A) * (1 / pi)): one rounding more)
// and PK_FDN (N / D) come from fast_div (v_rcp_f64, one Newton step, one residual correction)
// instead of IEEE divisions.  tests/test_plan_gpu.py::test_hop_words_vs_dense_records measures the
// device words against the dense records (within a few ulps, 1e-15 relative).
AFS_HD inline uint64_t plan_word_fast(uint32_t kind, const double *p, double ratio) {
#if defined(__HIP_DEVICE_COMPILE__)
  double x, y;
  {
#pragma clang fp contract(off)
    const double r1 = 1.0 - ratio;
    x = r1 * p[0] + ratio * p[1];
    y = r1 * p[2] + ratio * p[3];
  }
  const double a = at_least(at_least(x, AMIN), 0.1);
  const bool invd = kind == PK_INVD, fdn = kind == PK_FDN;
  // (a constant word's inputs are no area: its lane computes on them and discards the value)
  const double s = fast_sqrt(invd ? (4.0 * a) * (1.0 / PI) : a);
  const double q = fast_div(fdn ? x : 1.0, fdn ? y : (invd ? s : a));
  const double v = kind == PK_SQRT ? s : q;
  return kind == PK_CONST ? plan_bits(p[0]) : plan_bits(v);
#else
  return plan_word_eval(kind, p, ratio);
#endif
}

// The double at LDS byte offset b of an utterance block (SecRec / ArmRec fields).
AFS_HD inline double &xat(double *X, uint32_t b) { return *reinterpret_cast<double *>(reinterpret_cast<char *>(X) + b); }
AFS_HD inline const double &xat(const double *X, uint32_t b) {
  return *reinterpret_cast<const double *>(reinterpret_cast<const char *>(X) + b);
}

// Lane registers.
// Only the persistent state and the frame cache live here; per-sample intermediates
// go through the LDS block or are recomputed from unchanged state.
template <int W>
struct Lane {
  using S = Shape<W>;
  double p[S::NSL], pr[S::NSL], w[S::NSL], wr[S::NSL], wr2[S::NSL];  // sections
  double u[S::NSL], ur[S::NSL], un[S::NSL];                          // their in-currents
  double aL[S::ND], aR[S::ND], lL[S::ND], lR[S::ND];                 // frame cache
  double al[S::ND], be[S::ND];                                        // dynamic wall terms
  double damp[S::NDP], dout[S::NDP], dcut[S::NDP];                   // dipoles gl + k W
  double rad_u[2];                                                    // owner of 64 / 83: radiation currents' old u
  double sample;                                                     // lane 0
  uint64_t planw;                                                    // word gl of this sample's plan (tree_plan.h)
  uint32_t racc[S::NDP];                                             // rand() sums of owned dipoles
  uint32_t rtmp[8];                                                  // rand() block scratch
  int32_t rhead, rpend;                                              // rand() ring head, values pending (rng_ring_seed)
  ArmCarry ac;                                                       // arm solver, during the solve
  // per-sample values of the geometry/network block (not state: cleared before a save)
  double acur[S::ND], lcur[S::ND];                                   // area, length of the slots
  double anx[S::ND], apv[S::ND];                                     // areas of sections s+1, s-1
};

// Cross-lane collectives every execution policy provides (results are uniform over the W
// lanes of one utterance):
//   x.ballot(f)     -> uint64_t with bit gl = f(gl, R)
//   x.min_index(f)  -> the smallest MinIdx::v of f(gl, R), ties to the smallest index
//   x.max_value(f)  -> the largest f(gl, R) under strict ">" (a NaN never wins)
struct MinIdx { double v; int i; };
// x.dyn_neighbors(): R.anx[j] / R.apv[j] = R.acur of the owners of dynamic sections s+1 / s-1
// (s = the section of slot j; lanes' values as the interpolation left them).
// x.scan_add<N>(f, g): f(gl, R) -> U4; inclusive prefix sums (mod 2^32) of the first N
// components over lanes 0..gl are handed to g(gl, R, sums).
// x.pull<K, N>(f, g): f(gl, R) -> D4; g(gl, R, v) gets the first N components of lane gl+K's
// value (zeros when gl+K is outside the lane's group of 16: one DPP row on the device).
struct U4 { uint32_t v[4]; };
AFS_HD inline MinIdx min_idx_combine(MinIdx a, MinIdx b) {
  return (b.v < a.v || (b.v == a.v && b.i < a.i)) ? b : a;
}
AFS_HD inline double max_combine(double a, double b) { return (b > a) ? b : a; }

template <int W>
AFS_HD inline int slot_section(int j, int gl) {
  return j < Shape<W>::ND ? dyn_section(W, j, gl) : static_section(W, j - Shape<W>::ND, gl);
}

// ---------------------------------------------------------------------------
// math helpers
// ---------------------------------------------------------------------------
// The section-area clamp (Tube.cpp:337).  clampA keeps a NaN (the reference's comparison does, and
// a NaN frame area must give NaN audio from its transition on); clampA_num is at_least for the
// per-sample areas whose NaN reaches the audio by another path as well: the interpolated pharynx /
// mouth areas (a NaN frame area also makes that section's frame length NaN, frame_load, so the
// interpolated length carries it into the system in the same sample) and the glottis areas (a NaN
// there comes from NaN pressures, already in the system).
AFS_HD inline double clampA(double a) { return a < AMIN ? AMIN : a; }
AFS_HD inline double clampA_num(double a) { return at_least(a, AMIN); }
// A frame's section length, NaN when the section's area is (see clampA_num).
AFS_HD inline double frame_length(double area, double length) { return area != area ? area : length; }

AFS_HD inline double glottis_q(double f0) {
  double q = 1.0 + (f0 - G_NAT_F0) * (1.0 / G_F0_DIV_Q);
  return at_least(q, 0.05);
}

// getOpenCloseDimensions (TriangularGlottis.cpp:474-576), as selects (the three cases and the
// apex test are evaluated and chosen; no branch splits the geometry block)
AFS_HD inline void glottis_open_close_one(double rest, double cord, double rel, double &olen, double &clen,
                                          double &ow, double &cz) {
  const double back = rest + rel;
  const double front = (rest < 0.0) ? back : rel;
  const bool open = back > 0.0 && front > 0.0;
  const bool closed = back <= 0.0 && front <= 0.0;
  double r = rest;
  if (fabs(r) < 0.000000001) r = 0.000000001;
  const double apex = cord * (1.0 + fast_div(rel, r));
  const bool part = !open && !closed && apex >= 0.0 && apex <= cord;
  const bool pb = part && back > 0.0, pf = part && !(back > 0.0);
  olen = open ? cord : pb ? apex : pf ? cord - apex : 0.0;
  ow = open ? back + front : pb ? back : pf ? front : 0.0;
  clen = open ? 0.0 : pb ? cord - apex : pf ? apex : cord;
  cz = open ? 0.0 : pb ? 0.5 * (apex + cord) : pf ? 0.5 * apex : 0.5 * cord;
}
AFS_HD inline void glottis_open_close(const double *gp, double cord, double rel0, double rel1,
                                      double *olen, double *clen, double *ow, double *cz) {
  glottis_open_close_one(gp[2], cord, rel0, olen[0], clen[0], ow[0], cz[0]);
  glottis_open_close_one(gp[3], cord, rel1, olen[1], clen[1], ow[1], cz[1]);
}

// Gain of the glottis dipole source, 0.5e-7 * 10^(aspiration dB / 20) (TdsModel.cpp:1546),
// evaluated with the glottis (off the constriction phase's chains).
AFS_HD inline double glottis_dipole_gain(double aspiration_db) {
  return 0.5e-7 * exp(aspiration_db * (2.302585092994045684 / 20.0));
}

// Areas and lengths of the two glottis sections (23, 24) for the network phase.
struct GlotOut { double a0, a1, l0, l1; };

// TwoMassModel::calcGeometry / getTubeData (TwoMassModel.cpp:359-440) and incTime (:157-349)
// from the interpolated controls gp, the pressures p4 = p[22..25] of the previous sample and the
// relative displacements rel (current 0/1, previous 2/3, as for the triangular glottis); the new
// displacements go to rel_out.
template <class CT>
AFS_HD inline GlotOut two_mass_glottis(const CT &C, const double *gp, const double *p4, const double *rel,
                                       double *rel_out) {
  double Q = 1.0 + (gp[0] - TM_NAT_F0) * (1.0 / TM_F0_DIV_Q);  // getTensionParameter (:467-485)
  Q = at_least(Q, 0.05);
  const double f = fast_sqrt(Q), inv_f = fast_rcp(f), inv_q = fast_rcp(Q);
  const double len = TM_REST_LEN * f, th0 = TM_REST_THICK0 * inv_f, th1 = TM_REST_THICK1 * inv_f;
  const double rel0 = rel[0], rel1 = rel[1];
  const double rest0 = gp[2], rest1 = gp[3];
  // geometry
  double a0 = rest0 + rel0, a1 = rest1 + rel1;
  const double ab0 = a0, ab1 = a1;  // incTime's absolute displacements are not clipped
  a0 = nonneg(a0);
  a1 = nonneg(a1);
  double passive = 2.0 * rest1;
  passive = nonneg(passive);
  double chink = passive * TM_CHINK_LEN + gp[4];
  chink = nonneg(chink);
  GlotOut go{clampA_num(2.0 * len * a0 + chink), clampA_num(2.0 * len * a1 + chink), th0, th1};
  // incTime
  const double crit = 0.5 * TM_CRIT_WIDTH;
  const double min0 = crit - rest0, min1 = crit - rest1;
  const double m0 = TM_MASS0 * inv_q, m1 = TM_MASS1 * inv_q;
  const double k0 = TM_K0 * Q, k1 = TM_K1 * Q;
  double ck0 = TM_KC0 * Q, ck1 = TM_KC1 * Q, ce0 = TM_CETA0, ce1 = TM_CETA1;
  const double kc = TM_KCOUPLE * Q * Q;
  const double df = gp[5];
  double dr0 = TM_DAMP0, dr1 = TM_DAMP1;
  if (ab0 <= crit) dr0 += 1.0;
  if (ab1 <= crit) dr1 += 1.0;
  const double r0 = 2.0 * dr0 * fast_sqrt(m0 * k0) * df * df, r1 = 2.0 * dr1 * fast_sqrt(m1 * k1) * df * df;
  const double p0 = p4[0], p1 = p4[1], p2 = p4[2], p3 = p4[3];
  const bool open0 = ab0 > TM_CRIT_WIDTH, open1 = ab1 > TM_CRIT_WIDTH;
  const double fp0 = open0 ? p1 : p0;
  const double fp1 = open1 ? p2 : (open0 ? p1 : p3);
  const double fo0 = fp0 * len * th0, fo1 = fp1 * len * th1;
  if (rel0 > min0) { ck0 = 0.0; ce0 = 0.0; }
  if (rel1 > min1) { ck1 = 0.0; ce1 = 0.0; }
  const double d0 = rel0 - min0, d1 = rel1 - min1;
  const double nl0 = k0 * TM_ETA0 * rel0 * rel0 * rel0 + ck0 * ce0 * d0 * d0 * d0;
  const double nl1 = k1 * TM_ETA1 * rel1 * rel1 * rel1 + ck1 * ce1 * d1 * d1 * d1;
  const double T = C.h.Tt;
  const double A = m0 + r0 * T + T * T * (k0 + ck0) + kc * T * T;
  const double B = -kc * T * T;
  const double Cq = -kc * T * T;
  const double D = m1 + r1 * T + T * T * (k1 + ck1) + kc * T * T;
  const double E = fo0 * T * T + 2.0 * m0 * rel0 - m0 * rel[2] + r0 * T * rel0 + T * T * ck0 * min0 - nl0 * T * T;
  const double F = fo1 * T * T + 2.0 * m1 * rel1 - m1 * rel[3] + r1 * T * rel1 + T * T * ck1 * min1 - nl1 * T * T;
  double det = A * D - B * Cq;
  if (fabs(det) < 0.000000001) det = 0.000000001;
  const double inv_det = fast_rcp(det);
  rel_out[2] = rel0;
  rel_out[3] = rel1;
  rel_out[0] = (E * D - B * F) * inv_det;
  rel_out[1] = (A * F - E * Cq) * inv_det;
  return go;
}

// getGlottalEntranceLossCoeffFlucher2011(pressure, d) (TdsModel.cpp:1048-1092)
AFS_HD inline double fulcher_kent(double pressure_dPa, double d_cm) {
  double pc = pressure_dPa / 979.7;
  double D = d_cm;
  if (pc < 0.001) pc = 0.001;
  if (D < 0.001) D = 0.001;
  const double logD = log10(D);
  const double a = pow(10.0, 0.7953 * logD * logD + 1.4741 * logD + 0.6529);
  const double b = -0.7427 * logD * logD + -1.6209 * logD + -0.875;
  double k = a * pow(pc, b);
  if (k < 0.6) k = 0.6;
  if (k > 18.0) k = 18.0;
  return k;
}

// getJunctionInductance (TdsModel.cpp:1745-1778) from the inverse radii sqrt(pi / A) of the two
// sections, which the network phase computed already (X_RAD): with a, b the larger and the
// smaller radius, 8 rho H / (3 pi^2 b) and H = 1 - b / a give 8 rho / (3 pi^2) (1/b - 1/a).  The
// areas are >= MIN_AREA (the reference's clamps are no-ops).
AFS_HD inline double junction_l(double ir1, double ir2) {
  return (8.0 * RHO / (3.0 * PI * PI)) * fabs(ir1 - ir2);
}

// IirFilter::getOutputSample on a shift-register state x[0..n-1], y[0..n-1] (newest first).
// State and coefficients are read into registers first (one batch of loads), the shifted
// state is written back with independent stores.
template <int N>
AFS_HD inline double iir_run(double *st, const double *a, const double *b, double x) {
  double sx[N], sy[N], ca[N + 1], cb[N + 1];
#pragma unroll
  for (int k = 0; k < N; ++k) { sx[k] = st[k]; sy[k] = st[N + k]; }
#pragma unroll
  for (int k = 0; k <= N; ++k) { ca[k] = a[k]; cb[k] = b[k]; }
  AFS_SCHED_BARRIER();
  double acc = ca[0] * x;
#pragma unroll
  for (int k = 1; k <= N; ++k) {
    acc += ca[k] * sx[k - 1];
    acc += cb[k] * sy[k - 1];
  }
  st[0] = x;
  st[N] = acc;
#pragma unroll
  for (int k = 1; k < N; ++k) { st[k] = sx[k - 1]; st[N + k] = sy[k - 1]; }
  return acc;
}

AFS_HD inline int32_t rng_next(int32_t *r) {
  int f = r[31];
  int q = f - 3;
  if (q < 0) q += 31;
  uint32_t v = (uint32_t)r[f] + (uint32_t)r[q];
  r[f] = (int32_t)v;
  r[31] = (f + 1 == 31) ? 0 : f + 1;
  return (int32_t)(v >> 1);
}

// glibc __srandom_r: Schrage fill + 310 discarded outputs
AFS_HD inline void rng_seed(int32_t *r, uint32_t seed) {
  if (seed == 0) seed = 1;
  int32_t word = (int32_t)seed;
  r[0] = word;
  for (int i = 1; i < 31; ++i) {
    long long hi = word / 127773;
    long long lo = word % 127773;
    long long nw = 16807 * lo - 2836 * hi;
    if (nw < 0) nw += 2147483647;
    word = (int32_t)nw;
    r[i] = word;
  }
  r[31] = 3;
  for (int k = 0; k < 310; ++k) (void)rng_next(r);
}

// The rand() stream as a sequence r_i = r_{i-3} + r_{i-31} (mod 2^32), output r_i >> 1 --
// glibc's TYPE_3 generator read in generation order.  The LDS block holds the last 64
// values (RNG_R, index = sequence number mod 64: the generator's 31-value history and a
// block), the inclusive prefix sums of the outputs S_i = sum_{i' <= i} (r_i' >> 1) (RNG_S,
// index = sequence number mod RNG_SRING; sums of draws are differences of two of them),
// and in the lane registers (Lane::rhead, Lane::rpend, the same on every lane of the utterance:
// no LDS round trip before the noise phase's addresses) the sequence number mod RNG_SRING of the
// next value to generate and how many generated values have not been drawn yet (rng_ahead).
// (AFS_RNG_AHEAD: see the top of this file)
constexpr int RNG_RING = 64, RNG_SRING = AFS_RNG_AHEAD >= 2 ? 128 : 64;
constexpr int RNG_R = 0, RNG_S = RNG_RING;
static_assert((RNG_S + RNG_SRING) / 2 == X_GP - X_RNG, "the rand() region of the LDS block");
// values per generation block: 3 residue chains x min(W, 10) lanes (<= 30 keeps every
// term of the block in the 31-value history)
template <int W> constexpr int rng_lanes() { return W < 10 ? W : 10; }

// Ring after srand(seed): the 31 most recent values in generation order at 0..30.
AFS_HD inline void rng_ring_seed(uint32_t *g, uint32_t seed) {
  int32_t st[32];
  rng_seed(st, seed);
  const int f = st[31];  // glibc's fptr: the oldest value of the window
  for (int j = 0; j < RNG_S + RNG_SRING; ++j) g[j] = 0;
  for (int j = 0; j < 31; ++j) g[RNG_R + j] = (uint32_t)st[(f + j) % 31];
  // (the head, 31 -- S[30] = 0 is the base of the prefix sums -- and the pending count 0: reset_lane)
}

// ---------------------------------------------------------------------------
// Reset (Synthesizer::reset + TdsModel::resetMotion + TriangularGlottis::resetMotion)
// ---------------------------------------------------------------------------
template <int W>
AFS_HD inline void reset_lane(int gl, Lane<W> &R) {
  using S = Shape<W>;
  (void)gl;
#pragma unroll
  for (int j = 0; j < S::NSL; ++j) {
    R.p[j] = R.pr[j] = R.w[j] = R.wr[j] = R.wr2[j] = 0.0;
    R.u[j] = R.ur[j] = R.un[j] = 0.0;
  }
#pragma unroll
  for (int j = 0; j < S::ND; ++j) {
    R.aL[j] = R.aR[j] = R.lL[j] = R.lR[j] = R.al[j] = R.be[j] = 0.0;
  }
  R.planw = 0;
#pragma unroll
  for (int k = 0; k < S::NDP; ++k) { R.damp[k] = 0.0; R.dout[k] = 0.0; R.dcut[k] = 3000.0; }
  for (int k = 0; k < 2; ++k) R.rad_u[k] = 0.0;
  R.sample = 0.0;
#pragma unroll
  for (int k = 0; k < S::NDP; ++k) R.racc[k] = 0u;
  R.rhead = 31;
  R.rpend = 0;
}

AFS_HD inline void reset_lds(double *X, uint32_t seed) {
  for (int k = 0; k < X_TOTAL; ++k) X[k] = 0.0;
  rng_ring_seed((uint32_t *)(X + X_RNG), seed);
}

// ---------------------------------------------------------------------------
// Frame transition: cache the two frames of the interpolation.
// ---------------------------------------------------------------------------
template <int W>
AFS_HD inline void frame_load(int gl, Lane<W> &R, double *X, const afs_frame *fl, const afs_frame *fr) {
  using S = Shape<W>;
#pragma unroll
  for (int j = 0; j < S::ND; ++j) {
    int s = dyn_section(W, j, gl);
    int m = s - S_PHARYNX0;
    if (m >= 0 && m < NPM) {
      R.aL[j] = clampA(fl->area_cm2[m]);   // the caller's Tube stores clamped areas (Tube.cpp:337)
      R.aR[j] = clampA(fr->area_cm2[m]);
      R.lL[j] = frame_length(fl->area_cm2[m], fl->length_cm[m]);
      R.lR[j] = frame_length(fr->area_cm2[m], fr->length_cm[m]);
    }
  }
  // (laterality, articulators and teeth position only steer the noise sources: tree_plan.h)
  if (gl == 0) {
    X[X_FRAME + 0] = fl->teeth_position_cm;
    X[X_FRAME + 1] = fr->teeth_position_cm;
    X[X_FRAME + 2] = clampA(fl->velum_opening_cm2);   // getVelumOpening = clamped noseSection[0]
    X[X_FRAME + 3] = clampA(fr->velum_opening_cm2);
    for (int k = 0; k < 6; ++k) {
      X[X_FRAME + 4 + k] = fl->glottis[k];
      X[X_FRAME + 10 + k] = fr->glottis[k];
    }
  }
}

// The fields of a frame that frame_load reads, loaded ahead (tree_kernel.h, dense kernel):
// the areas / lengths of the lane's pharynx/mouth slots and the frame-rate values.
template <int W>
struct NextFrame {
  double a[Shape<W>::ND], l[Shape<W>::ND], x[8];  // x: teeth, velum, glottis[6]
  AFS_HD void load(int gl, const afs_frame *f) {
#pragma unroll
    for (int j = 0; j < Shape<W>::ND; ++j) {
      const int m = dyn_section(W, j, gl) - S_PHARYNX0;
      const int mm = (m >= 0 && m < NPM) ? m : 0;  // (other slots load section 25's and discard it)
      a[j] = f->area_cm2[mm];
      l[j] = f->length_cm[mm];
    }
    x[0] = f->teeth_position_cm;
    x[1] = f->velum_opening_cm2;
    for (int k = 0; k < 6; ++k) x[2 + k] = f->glottis[k];
  }
};
// frame_load(fr, next) when fr was the previous transition's right frame: the right frame
// becomes the left one, the right one comes from the loaded fields (the same values frame_load
// gives).
template <int W>
AFS_HD inline void frame_shift(int gl, Lane<W> &R, double *X, const NextFrame<W> &nf) {
  using S = Shape<W>;
#pragma unroll
  for (int j = 0; j < S::ND; ++j) {
    const int m = dyn_section(W, j, gl) - S_PHARYNX0;
    if (m >= 0 && m < NPM) {
      R.aL[j] = R.aR[j];
      R.lL[j] = R.lR[j];
      R.aR[j] = clampA(nf.a[j]);
      R.lR[j] = frame_length(nf.a[j], nf.l[j]);
    }
  }
  if (gl == 0) {
    X[X_FRAME + 0] = X[X_FRAME + 1];
    X[X_FRAME + 1] = nf.x[0];
    X[X_FRAME + 2] = X[X_FRAME + 3];
    X[X_FRAME + 3] = clampA(nf.x[1]);
    for (int k = 0; k < 6; ++k) {
      X[X_FRAME + 4 + k] = X[X_FRAME + 10 + k];
      X[X_FRAME + 10 + k] = nf.x[2 + k];
    }
  }
}

// ---------------------------------------------------------------------------
// Phase G: tube interpolation (all lanes) and the glottis (lane 0).
// ---------------------------------------------------------------------------
template <int W>
AFS_HD inline void phase_interpolate(int gl, Lane<W> &R, double *X, const Consts &C, double ratio) {
  // Branch-free over the lane's slots: pharynx/mouth sections interpolate area, length and
  // laterality, the nose sections 65..68 take the velum taper (Tube.cpp:402-416); other slots
  // (glottis, absent) compute on stand-ins.  The area and length stay in the lane (acur,
  // lcur) for the network phase of the same block.  (The constriction scans that read the
  // interpolated geometry of all sections run ahead of the time loop: tree_plan.h.)  Not
  // contracted into fmas: K5 (tree_plan.h PlanGeom) evaluates the same products and sums, and
  // the reference's own a * (1 - r) + b * r rounds each product.
#pragma clang fp contract(off)
  using S = Shape<W>;
  (void)gl;
  (void)X;
  const double r1 = 1.0 - ratio;
  const double open = r1 * X[X_FRAME + 2] + ratio * X[X_FRAME + 3];
#pragma unroll
  for (int j = 0; j < S::ND; ++j) {
    const int k = j * W + gl;
    const int s = DYN0 + k;
    const bool pm = s >= S_PHARYNX0 && s <= S_LAST_MOUTH;
    const bool nose = s >= S_NOSE0 && k < NDYNS;
    const double apm = r1 * R.aL[j] + ratio * R.aR[j];
    const double lpm = r1 * R.lL[j] + ratio * R.lR[j];
    const int i = s - S_NOSE0;
    const double anose = open + ((double)(i * i) * (C.h.nose4_area - open)) * (1.0 / 16);
    // (both candidates clamped: one clamp after the select measured -0.2 %, profiles/r03x_ab.txt)
    const double a = pm ? clampA_num(apm) : (nose ? clampA(anose) : 1.0);
    R.acur[j] = a;
    R.lcur[j] = pm ? lpm : C.h.len_nose0;
  }
}

// The glottis of one sample (lane-uniform inputs: every lane of the utterance computes the same
// values, see Exec::par_uniform): calcGeometry at the interpolated controls with the current
// displacements, then incTime with the pressures p4 = p[22..25] of the previous sample.  In
// three steps -- the loads (glottis_inputs), the arithmetic (glottis_eval), the stores
// (glottis_commit) -- so that the block can issue every load before its first store and the
// glottis chain interleaves with the network (an LDS load after a store to the same block
// cannot be moved above it).
struct GlotIn { double fl[6], fr[6], rel[4]; };
struct GlotRes { GlotOut go; double gp[6], rel[4]; };

AFS_HD inline GlotIn glottis_inputs(const double *X, int relx = X_RELX) {
  GlotIn in;
  for (int k = 0; k < 6; ++k) {
    in.fl[k] = X[X_FRAME + 4 + k];
    in.fr[k] = X[X_FRAME + 10 + k];
  }
  for (int k = 0; k < 4; ++k) in.rel[k] = X[relx + k];
  return in;
}

template <int MODEL, class CT>
AFS_HD inline GlotRes glottis_eval(const GlotIn &in, const CT &C, double ratio, const double *p4) {
  const double r1 = 1.0 - ratio;
  GlotRes res;
  double *gp = res.gp;
  {  // (uncontracted as Tube::interpolate and K5's aspiration strength, tree_plan.h)
#pragma clang fp contract(off)
    for (int k = 0; k < 6; ++k) gp[k] = r1 * in.fl[k] + ratio * in.fr[k];
  }
  if constexpr (MODEL == AFS_GLOTTIS_TWO_MASS) {
    res.go = two_mass_glottis(C, gp, p4, in.rel, res.rel);
    gp[5] = GLOTTIS_DEFAULT_ASPIRATION_DB;  // X_GP + 5 is read as the aspiration strength
    return res;
  } else {
    const double rel0 = in.rel[0], rel1 = in.rel[1];
    // calcGeometry + getTubeData + Tube::setGlottisGeometry (TriangularGlottis.cpp:338-411)
    // (divisions sharing a denominator use one reciprocal; sqrt(m k) is a constant since
    // m ~ 1/q and k ~ q)
    double chink = nonneg(gp[4]);
    double q = glottis_q(gp[0]);
    double f = fast_sqrt(q);
    const double inv_f = fast_rcp(f), inv_q = fast_rcp(q);
    double cord = G_REST_LEN * f;
    const double inv_cord = fast_rcp(cord);
    double th0 = G_REST_THICK0 * inv_f, th1 = G_REST_THICK1 * inv_f;
    double olen[2], clen[2], ow[2], cz[2];
    glottis_open_close(gp, cord, rel0, rel1, olen, clen, ow, cz);
    res.go = GlotOut{clampA_num(olen[0] * ow[0] + chink), clampA_num(olen[1] * ow[1] + chink), th0, th1};
    // incTime (TriangularGlottis.cpp:154-330) with the previous sample's pressures
    const double Tt = C.h.Tt;
    const double p0 = p4[0], p1 = p4[1], p2 = p4[2], p3 = p4[3];
    double m0 = G_MASS0 * inv_q, m1 = G_MASS1 * inv_q;
    double al0 = clen[0] * inv_cord, al1 = clen[1] * inv_cord;
    double k0 = G_K0 * q, k1 = G_K1 * q, kc0 = G_KC0 * q, kc1 = G_KC1 * q;
    double kcp = G_KCOUPLE * q * q;
    double dr0 = G_DAMP0 + al0 * 1.0, dr1 = G_DAMP1 + al1 * 1.0;
    double rr0 = 2.0 * dr0 * C.h.g_smk0, rr1 = 2.0 * dr1 * C.h.g_smk1;
    double fo0 = p1 * olen[0] * th0;
    double fo1 = p2 * olen[1] * th1;
    fo0 += 0.5 * 0.5 * (p0 + p1) * G_INLET * cord;
    fo1 += 0.5 * 0.5 * (p3 + p2) * G_OUTLET * cord;
    double rs0 = (gp[2] >= 0.0) ? gp[2] * (1.0 - cz[0] * inv_cord) : gp[2];
    double rs1 = (gp[3] >= 0.0) ? gp[3] * (1.0 - cz[1] * inv_cord) : gp[3];
    double A = m0 + rr0 * Tt + Tt * Tt * (k0 + kc0 * al0) + kcp * Tt * Tt;
    double B = -kcp * Tt * Tt;
    double Cq = -kcp * Tt * Tt;
    double Dq = m1 + rr1 * Tt + Tt * Tt * (k1 + kc1 * al1) + kcp * Tt * Tt;
    double Ee = fo0 * Tt * Tt + 2.0 * m0 * rel0 - m0 * in.rel[2] + rr0 * Tt * rel0 - Tt * Tt * kc0 * al0 * rs0;
    double Ff = fo1 * Tt * Tt + 2.0 * m1 * rel1 - m1 * in.rel[3] + rr1 * Tt * rel1 - Tt * Tt * kc1 * al1 * rs1;
    double det = A * Dq - B * Cq;
    if (fabs(det) < 0.000000001) det = 0.000000001;
    const double inv_det = fast_rcp(det);  // |det| >= 1e-9
    res.rel[2] = rel0;
    res.rel[3] = rel1;
    res.rel[0] = (Ee * Dq - B * Ff) * inv_det;
    res.rel[1] = (A * Ff - Ee * Cq) * inv_det;
    return res;
  }
}

// The triangular glottis with its two masses on the two halves of an utterance's 16 lanes
// (device; the CPU emulator runs glottis_eval): every lane evaluates the shared terms, lanes
// 0-7 mass 0 and lanes 8-15 mass 1 with the operations glottis_eval applies to that mass (its
// constants from the tables' gmass row), and each mass's area, A and E terms reach the other
// half by a row rotation by 8 (xch): ~140 fewer instructions per sample, +1.1 % (A/B,
// profiles/r03ag_ab.txt).  The same operations as glottis_eval; under the kernel's fma
// contraction the compiler may fuse a few of them differently than in the uniform form (the
// parity figures move in their third digit).
template <class CT, class XCH>
AFS_HD inline GlotRes glottis_eval_split(const GlotIn &in, const CT &C, double ratio, const double *p4, int h,
                                         XCH xch) {
  const double r1 = 1.0 - ratio;
  GlotRes res;
  double *gp = res.gp;
  {
#pragma clang fp contract(off)
    for (int k = 0; k < 6; ++k) gp[k] = r1 * in.fl[k] + ratio * in.fr[k];
  }
  const double rel0 = in.rel[0], rel1 = in.rel[1];
  double chink = nonneg(gp[4]);
  double q = glottis_q(gp[0]);
  double f = fast_sqrt(q);
  const double inv_f = fast_rcp(f), inv_q = fast_rcp(q);
  double cord = G_REST_LEN * f;
  const double inv_cord = fast_rcp(cord);
  double th0 = G_REST_THICK0 * inv_f, th1 = G_REST_THICK1 * inv_f;
  const bool m1 = h != 0;
  const double *K = C.h.gmass[m1 ? 1 : 0];
  const double rest = m1 ? gp[3] : gp[2], rel = m1 ? rel1 : rel0, relp = m1 ? in.rel[3] : in.rel[2];
  double olen, clen, ow, cz;
  glottis_open_close_one(rest, cord, rel, olen, clen, ow, cz);
  const double area = clampA_num(olen * ow + chink);
  const double th = K[6] * inv_f;
  const double Tt = C.h.Tt;
  const double p0 = p4[0], p1 = p4[1], p2 = p4[2], p3 = p4[3];
  double m = K[0] * inv_q;
  double al = clen * inv_cord;
  double k = K[1] * q, kc = K[2] * q;
  double kcp = G_KCOUPLE * q * q;
  double dr = K[3] + al * 1.0;
  double rr = 2.0 * dr * K[4];
  double fo = (m1 ? p2 : p1) * olen * th;
  fo += 0.5 * 0.5 * ((m1 ? p3 : p0) + (m1 ? p2 : p1)) * K[5] * cord;
  double rs = (rest >= 0.0) ? rest * (1.0 - cz * inv_cord) : rest;
  double Am = m + rr * Tt + Tt * Tt * (k + kc * al) + kcp * Tt * Tt;
  double Em = fo * Tt * Tt + 2.0 * m * rel - m * relp + rr * Tt * rel - Tt * Tt * kc * al * rs;
  const double oa = xch(area), oA = xch(Am), oE = xch(Em);
  res.go = GlotOut{m1 ? oa : area, m1 ? area : oa, th0, th1};
  const double A = m1 ? oA : Am, Dq = m1 ? Am : oA, Ee = m1 ? oE : Em, Ff = m1 ? Em : oE;
  double B = -kcp * Tt * Tt;
  double Cq = -kcp * Tt * Tt;
  double det = A * Dq - B * Cq;
  if (fabs(det) < 0.000000001) det = 0.000000001;
  const double inv_det = fast_rcp(det);
  res.rel[2] = rel0;
  res.rel[3] = rel1;
  res.rel[0] = (Ee * Dq - B * Ff) * inv_det;
  res.rel[1] = (A * Ff - Ee * Cq) * inv_det;
  return res;
}

// The upper mass's area of the triangular glottis this sample (go.a1 of glottis_eval_split: the
// same operations on its inputs), for the wave pairs' STAT wave, which needs no more of the glottis
// (AFS_PAIR_SPLIT1=2).
AFS_HD inline double glottis_upper_area(const GlotIn &in, double ratio) {
  const double r1 = 1.0 - ratio;
  double g0, g3, g4;
  {
#pragma clang fp contract(off)
    g0 = r1 * in.fl[0] + ratio * in.fr[0];
    g3 = r1 * in.fl[3] + ratio * in.fr[3];
    g4 = r1 * in.fl[4] + ratio * in.fr[4];
  }
  const double chink = nonneg(g4);
  const double q = glottis_q(g0);
  const double f = fast_sqrt(q);
  const double cord = G_REST_LEN * f;
  double olen, clen, ow, cz;
  glottis_open_close_one(g3, cord, in.rel[1], olen, clen, ow, cz);
  return clampA_num(olen * ow + chink);
}

// The glottis state of the sample: new displacements, interpolated controls (X_GP + 1, the lung
// pressure, is the row phase's source term of section 0).
AFS_HD inline void glottis_commit(double *X, const GlotRes &r, int relx = X_RELX) {
  for (int k = 0; k < 6; ++k) X[X_GP + k] = r.gp[k];
  for (int k = 0; k < 4; ++k) X[relx + k] = r.rel[k];
}

// ---------------------------------------------------------------------------
// Phase N: per-section network elements L, C, R, wall terms, D, E (TdsModel.cpp:732-1008).
// Static sections take L, C, R, alpha, E from the tables; only beta and D depend on state.
// ---------------------------------------------------------------------------
AFS_HD inline int static_index(int s) { return s < 23 ? s : s - 46; }

template <int W>
AFS_HD inline double static_beta(const Lane<W> &R, int j, const Uni &U, const Consts &C, int s) {
  const double *k = C.stat[static_index(s)];
  // (evaluated either way and selected: a branch here would split the slot block)
  const double v = k[ST_ALPHA] * (R.w[j] * k[ST_WC1] + R.wr[j] * k[ST_WC2] + R.wr2[j] * k[ST_LW] * (TH1 / TH));
  return U.opt.soft_walls ? v : 0.0;
}

template <int W, bool VARLOSS, int ROLE = ROLE_ALL>
AFS_HD inline void phase_network(int gl, Lane<W> &R, double *X, const Uni &U, const Consts &C, const GlotOut &go) {
  // One branch-free block over the lane's slots (absent slots compute on a valid section and
  // store into the sinks), so that the scheduler interleaves the slots' reciprocal and square
  // root chains; the glottal entrance (one section) and the transvelar source follow.
  using S = Shape<W>;
  const afs_options &opt = U.opt;
  const double dt = C.h.dt, idt = C.h.inv_dtTH, idt2 = C.h.inv_dt2TH2;
#pragma unroll
  for (int j = 0; j < S::NST; ++j) {
    const int jj = S::ND + j;
    if (!role_slot<ROLE>(jj, S::ND)) continue;
    const int s0 = static_section(W, j, gl);
    const int s = s0 < 0 ? 0 : s0;
    const double E = C.stat[static_index(s)][ST_E];
    const double beta = static_beta<W>(R, jj, U, C, s);
    X[X_D + (s0 < 0 ? NS : s)] = R.p[jj] + C.h.dtTH1 * R.pr[jj] - E * (beta - 0.0);  // (E: a table constant)
  }
  // Glottal entrance and transition terms of section 23 (TdsModel.cpp:898-950) with the
  // standard / van den Berg entrance loss: lane-uniform inputs (the flows into 23 and 24 are the
  // previous solution, the areas the glottis values), so every lane computes them inside the
  // block and slot 0 of lane 0 adds them; only lane 0 stores the separation state (the others
  // store into a sink).  The variable (Fulcher) loss keeps its lane-0 block after the loop.
  if constexpr (ROLE == ROLE_STAT) return;  // (the rest: the dynamic slots)
  double dR0g = 0.0, dR1g = 0.0;
  bool on0 = false, on1 = false;
  if constexpr (!VARLOSS) {
    const double kent = opt.glottis_loss == AFS_ENTRANCE_LOSS_VAN_DEN_BERG ? 1.375 : 1.0;
    double u23 = 0.0, u24 = 0.0;
    u23 += X[X_U + S_GLOT_LO];
    u24 += X[X_U + S_GLOT_UP];
    const double sa = C.h.area_last_trachea;
    dR0g = kent * 0.5 * RHO * fabs(u23) * (fast_rcp(go.a0 * go.a0) - fast_rcp(sa * sa));
    const double bt = (go.a1 < opt.flow_separation_area_ratio * go.a0) ? 1.0 : 0.0;
    const double gsep = 0.8 * X[X_GBF] + (1.0 - 0.8) * bt;
    X[gl == 0 ? X_GBF : X_ACT + 3] = gsep;
    dR1g = gsep * fabs(u24) * 0.5 * RHO * (fast_rcp(go.a1 * go.a1) - fast_rcp(go.a0 * go.a0));
    on0 = u23 > 0;
    on1 = u24 > 0;
  }
  double R0g = 0.0, R1g = 0.0, Eg[S::ND], betag[S::ND];
#pragma unroll
  for (int j = 0; j < S::ND; ++j) {
    const int k = j * W + gl;
    const bool present = k < NDYNS;
    if constexpr (S::ND * W > NDYP) {  // wider utterances (CPU emulator only): no sinks for all
      if (!present) continue;
    }
    const int s = present ? DYN0 + k : S_PHARYNX0;  // an absent slot computes on section 25
    const int ks = present ? k : NDYNS;             // and stores into the sinks
    const bool glot = (s == S_GLOT_LO || s == S_GLOT_UP);
    const bool pm = s >= S_PHARYNX0 && s <= S_LAST_MOUTH;
    // (from this block's interpolation and glottis; an absent slot has area and length 1)
    const double area = glot ? (s == S_GLOT_LO ? go.a0 : go.a1) : R.acur[j];
    const double len = glot ? (s == S_GLOT_LO ? go.l0 : go.l1) : R.lcur[j];
    // prepareTimeStep's section quantities (TdsModel.cpp:732-834), with the repeated
    // divisions folded into one reciprocal of the area and one of the wall surface.
    // (the divisions rewritten around one reciprocal of the area: the Poiseuille resistance of
    // the circular and the elliptic section (:741-760) as polynomials in 1/A, the wall terms with
    // the wall surface cancelled (alpha = surf / K, beta = k1 w + k2 w' + k3 w''); the decisions
    // -- elliptic or not, the surface clamp -- are the reference's comparisons)
    const double inv_area = fast_rcp(area);
    const double r0 = fast_sqrt(area * (1.0 / PI));
    const double ia2 = inv_area * inv_area;
    const bool ell = r0 < (glot ? 0.8 : 1.6);
    // elliptic: 2 mu len (a^2 + b^2) / (pi a^3 b^3), a = rmin, b = A / (pi rmin)
    //         = len / A (2 mu pi^2 rmin^2 / A^2 + 2 mu / rmin^2); circular: 4 mu pi len / A^2
    const double ce = glot ? 2.0 * MU * PI * PI * 0.64 : 2.0 * MU * PI * PI * 2.56;
    const double cf = glot ? 2.0 * MU / 0.64 : 2.0 * MU / 2.56;
    const double Rr = ell ? (len * inv_area) * fma(ce, ia2, cf) : (4.0 * MU * PI * len) * ia2;
    const double L = (RHO * 0.5 * len) * inv_area;
    const double Cc = (area * len) * (1.0 / (RHO * CSND * CSND));
    double surf = (2.0 * PI * r0) * len;
    surf = at_least(surf, AMIN);
    const bool walls = opt.soft_walls && !glot;
    const double alpha = walls ? surf * C.h.wall_invK : 0.0;
    const double beta = walls ? fma(R.w[j], C.h.wall_k1, fma(R.wr[j], C.h.wall_k2, R.wr2[j] * C.h.wall_k3)) : 0.0;
    const double E = fast_div(dt * TH, Cc + alpha);
    (void)idt; (void)idt2;
    double R0 = Rr, R1 = Rr;
    // Bernoulli losses between pharynx/mouth sections (TdsModel.cpp:850-877)
    const bool turb = opt.turbulence_losses && pm;
    {  // pair (s, s+1)
      double u = 0.0;
      u += X[X_U + s + 1];
      const double Ai = R.anx[j];
      const bool on = turb && s < S_LAST_MOUTH && s != S_PHARYNX0 + 3 && s != S_LAST_PHARYNX;
      // (bitwise conditions and a select: with && / if, the compiler sinks the load of u into
      // a branch and waits for it there)
      const bool c = ((Ai < area) & (u > 0)) | ((Ai > area) & (u < 0));
      const double Rb = R1 - u * (0.5 * RHO) * ia2;
      R1 = (on & c) ? Rb : R1;
    }
    {  // pair (s-1, s)
      double u = 0.0;
      u += R.u[j];
      const double Aa = R.apv[j];
      const bool on = turb && s > S_PHARYNX0 && s - 1 != S_PHARYNX0 + 3 && s - 1 != S_LAST_PHARYNX;
      const bool c = ((area < Aa) & (u > 0)) | ((area > Aa) & (u < 0));
      const double Rb = R0 + u * (0.5 * RHO) * ia2;
      R0 = (on & c) ? Rb : R0;
    }
    if (j == (S_LAST_MOUTH - DYN0) / W) {  // the slot that holds section 64 on one lane
      // radiation resistance and inductance of the mouth (TdsModel.cpp:1874, 1889): 128 rho c /
      // (9 pi^2 A) and 8 rho / (3 pi sqrt(A pi)) = (8 rho / (3 pi)) r0 / A
      const double Rrad = C.h.rrad_c * inv_area;
      const double Lrad = (C.h.lrad_c * r0) * inv_area;
      const bool own = s == S_LAST_MOUTH;
      X[own ? X_RRAD : X_ACT] = Rrad;
      X[own ? X_RRAD + 1 : X_ACT + 1] = Lrad;
    }
    if (j == 0) {
      if constexpr (VARLOSS) {
        R0g = R0; R1g = R1;
      } else {  // section 23: the glottal entrance / transition terms
        const bool glo = s == S_GLOT_LO;
        R0 = (glo & on0) ? R0 + dR0g : R0;
        R1 = (glo & on1) ? R1 + dR1g : R1;
      }
    }
    Eg[j] = E;
    betag[j] = beta;
    // (carried in registers to the update: alpha through an LDS array and beta recomputed there
    // measured -2.1 %, profiles/r03ab_ab.txt)
    R.al[j] = alpha;
    R.be[j] = beta;
    X[X_E + ks] = E;
    X[X_D + (present ? s : NS)] = R.p[j] + C.h.dtTH1 * R.pr[j] - E * (beta - 0.0);
    X[X_L + ks] = L;
    X[X_RAD + ks] = (PI * r0) * inv_area;  // 1 / r0 (the row phase's junction inductance)
    X[X_R0 + ks] = R0;
    X[X_R1 + ks] = R1;
  }
  if (VARLOSS && gl == S_GLOT_LO - DYN0) {  // glottal entrance and transition (TdsModel.cpp:898-950), slot 0
    const double area = go.a0;
    double R0 = R0g, R1 = R1g;
    double kent = 1.0;
    if (opt.glottis_loss == AFS_ENTRANCE_LOSS_VAN_DEN_BERG) {
      kent = 1.375;
    } else if (opt.glottis_loss == AFS_ENTRANCE_LOSS_VARIABLE) {  // :1019-1039
      const double tp = X[X_P4 + 0] - X[X_P4 + 3];
      kent = fulcher_kent(iir_run<4>(X + X_TGLOT, C.h.tglot_a, C.h.tglot_b, tp), area / 1.25);
    }
    double sa = C.h.area_last_trachea, ta = area;
    double u = 0.0;
    u += R.u[0];
    if (u > 0) R0 = R0 + kent * 0.5 * RHO * fabs(u) * (fast_rcp(ta * ta) - fast_rcp(sa * sa));
    sa = ta;
    ta = go.a1;
    double bt = (ta < opt.flow_separation_area_ratio * sa) ? 1.0 : 0.0;
    double g = 0.8 * X[X_GBF] + (1.0 - 0.8) * bt;
    X[X_GBF] = g;
    u = 0.0;
    u += X[X_U + S_GLOT_UP];
    if (u > 0) R1 = R1 + g * fabs(u) * 0.5 * RHO * (fast_rcp(ta * ta) - fast_rcp(sa * sa));
    X[X_R0 + 0] = R0;
    X[X_R1 + 0] = R1;
  }
  constexpr int KTV = S_NOSE0 + 2 - DYN0, JTV = KTV / W, GTV = KTV % W;
  if (opt.transvelar_coupling && gl == GTV) {  // flow through the velum (:966-980, 996)
    double src = 0.0;
    src += iir_run<4>(X + X_TVEL, C.h.tone_a, C.h.tone_b, X[X_TVP]) +
           iir_run<4>(X + X_TVEL + 8, C.h.tvel2_a, C.h.tone_b, X[X_TVP + 1]);
    X[X_D + S_NOSE0 + 2] = R.p[JTV] + C.h.dtTH1 * R.pr[JTV] - Eg[JTV] * (betag[JTV] - src);
  }
}

// ---------------------------------------------------------------------------
// Phase T: dipole targets and amplitude smoothing (TdsModel.cpp:1456-1604, 1630-1643).
// The geometry half of calcNoiseSources -- which constrictions exist and which two dipole
// sources each drives with which weights -- comes from this sample's plan (tree_plan.h,
// computed ahead of the time loop).  What is left depends on the state: the flow through
// each narrowest section (the noise-smoothed flows of the previous sample), the particle
// velocity, the full amplitude and the cutoff.  Every lane evaluates the four constrictions
// (lane-uniform values) and keeps the targets of the dipoles it owns, in the reference's
// store order (glottis, tongue 1, tongue 2, lip; the downstream source after the upstream
// one), then smooths their amplitudes -- all inside the network block, no LDS round trip.
// ---------------------------------------------------------------------------
struct Target { uint32_t up; double tup, tdn, fc; bool on; };

// Noise-phase variants.  On most utterances only some constrictions ever exist and only some
// dipole sources are ever targeted -- static vowels: the glottis source alone (dipoles 2-4) on a
// third of them, the glottis and one tongue constriction below dipole 32 on another third -- yet
// the full phases evaluate all four constrictions and smooth, count and filter all NDP dipole
// slots of every lane at every sample.  A variant NZ evaluates the first NC constrictions (glottis,
// tongue 1, tongue 2, lip) and processes the first NS slots; K1 runs a launch's time loop for a
// wave in the lightest variant whose constrictions and dipole slots cover everything the launch's
// hop records say any of its samples may target (PlanHop::noise) and whose skipped slots hold no
// amplitude (damp == 0, so their smoother, filter and dipole samples stay exactly as they are: 0).
// The variants compute exactly the full phases' values (tree_kernel.h).  Ceiling measured with
// every wave forced into a variant, 8192 static vowels (profiles/r05b_noise_variant_ceiling_ab.txt):
// NZ 1 +4.8 %, NZ 2 +13 %.
// (heaviest first: the slot order's classes, tree_plan.h plan_noise_class16, use these values)
enum : int { NZ_FULL = 0, NZ_T1ALL = 1, NZ_TONGUE1 = 2, NZ_GLOTTIS = 3, NZ_COUNT = 4,
             NZ_DYN = -1 };  // NZ_DYN: the variant chosen at run time, in a phase of its own (sample_step)
// The variants compiled into the hop-mode kernel, a bit mask: 1 NZ_TONGUE1, 2 NZ_GLOTTIS,
// 4 NZ_T1ALL (each a whole copy of the kernel body: the instruction cache, shared by a CU pair,
// holds about one, so every variant costs the waves of the other variants on the same CUs;
// profiles/r05c_variants_ab.txt, r05d_variants_ab.txt)
#ifndef AFS_NZ_SET
#define AFS_NZ_SET 3
#endif
#define AFS_NZ_T1ALL ((AFS_NZ_SET & 4) != 0)
template <int W, int NZ>
struct NoiseV {
  static constexpr int NC = NZ == NZ_FULL ? 4 : (NZ == NZ_GLOTTIS ? 1 : 2);
  static constexpr int NS_ = (NZ == NZ_FULL || NZ == NZ_T1ALL) ? Shape<W>::NDP : (NZ == NZ_TONGUE1 ? 2 : 1);
  static constexpr int NS = NS_ < Shape<W>::NDP ? NS_ : Shape<W>::NDP;
  // PlanHop::noise bits this variant serves: constrictions 0 .. NC-1, dipoles below NS * W
  static constexpr uint64_t SERVES = (((1ull << NC) - 1) << NOISE_CON0) |
                                     (NS * W >= 64 ? ((1ull << NOISE_CON0) - 1) : ((1ull << (NS * W)) - 1));
};
static_assert(NoiseV<16, NZ_GLOTTIS>::SERVES == NOISE_SERVES16_GLOTTIS &&
                  NoiseV<16, NZ_TONGUE1>::SERVES == NOISE_SERVES16_TONGUE1 &&
                  NoiseV<16, NZ_T1ALL>::SERVES == NOISE_SERVES16_T1ALL,
              "tree_plan.h plan_noise_class16: the slot order's classes are the 16-lane variants");

AFS_HD inline double narrow_flow(const double *X, uint32_t o0, uint32_t o1) {
  double flow = 0.0;
  flow += xat(X, o0);  // (an absent output reads the zero slot)
  flow += xat(X, o1);
  return nonneg(flow);  // only outgoing flow (:1512-1517)
}

AFS_HD inline double clamp_fc(double fc) {
  return at_most(at_least(fc, 50.0), 2000.0);
}

template <int W, int NZ, class Xc>
AFS_HD inline void phase_targets(Xc &x, int gl, Lane<W> &R, const double *X, const Consts &C, double a_glot_up) {
  using V = NoiseV<W, NZ>;
  const uint64_t hdr = x.template rec<PW_HDR>(), uo = x.template rec<PW_UO>(), uol = x.template rec<PW_UOL>();
  const uint32_t fl = (uint32_t)hdr & 0xffu;
  Target t[4];
  {  // glottis: A = the upper glottis section's area (this sample's glottis), clamped at 0.1
    const SecRec &q = C.sec[S_GLOT_UP];
    const double A = at_least(a_glot_up, 0.1);
    const double v = narrow_flow(X, q.x_uo0, q.x_uo1) * fast_rcp(A);
    const double full = plan_double(x.template rec<PW_GAIN_G>()) * fabs(v) * v * v * fast_sqrt(A);
    const double fdn = plan_double(x.template rec<PW_FDN + 0>());
    t[0] = Target{(uint32_t)(hdr >> 8) & 0xffu, (1.0 - fdn) * full, fdn * full, 2000.0, (fl & PF_G) != 0};
  }
#pragma unroll
  for (int c = 0; c < V::NC - 1 && c < 2; ++c) {  // tongue constrictions: "normal" fricatives (:1547-1563)
    const uint32_t o = (uint32_t)(uo >> (32 * c));
    const double invA = plan_double(c ? x.template rec<PW_T2 + 0>() : x.template rec<PW_T1 + 0>());
    const double sqA = plan_double(c ? x.template rec<PW_T2 + 1>() : x.template rec<PW_T1 + 1>());
    const double invd = plan_double(c ? x.template rec<PW_T2 + 2>() : x.template rec<PW_T1 + 2>());
    const double fdn = plan_double(c ? x.template rec<PW_FDN + 2>() : x.template rec<PW_FDN + 1>());
    const double v = narrow_flow(X, o & 0xffffu, o >> 16) * invA;
    const double fc = 0.15 * v * invd;
    const double gain = (fl & (c ? PF_T2_TEETH : PF_T1_TEETH)) ? 10.0e-7 : 5.0e-7;
    double full = gain * fabs(v) * v * v * sqA;
    if (fl & (c ? PF_T2_LAT : PF_T1_LAT)) full = 0.0;
    t[1 + c] = Target{(uint32_t)(hdr >> (16 + 8 * c)) & 0xffu, (1.0 - fdn) * full, fdn * full, clamp_fc(fc),
                      (fl & (c ? PF_T2 : PF_T1)) != 0};
  }
  if constexpr (V::NC >= 4) {  // lower lip: flat spectrum, gain 2e-7 (:1523-1529)
    const double v = narrow_flow(X, (uint32_t)uol & 0xffffu, (uint32_t)(uol >> 16) & 0xffffu) *
                     plan_double(x.template rec<PW_L + 0>());
    const double full = 2.0e-7 * fabs(v) * v * v * plan_double(x.template rec<PW_L + 1>());
    const double fdn = plan_double(x.template rec<PW_FDN + 3>());
    t[3] = Target{(uint32_t)(hdr >> 32) & 0xffu, (1.0 - fdn) * full, fdn * full, 2000.0, (fl & PF_L) != 0};
  }
  // the owned dipoles: targets in store order, then the 40 Hz amplitude smoother
  // (branch-free over the slots; a slot past the 41 dipoles is never targeted and never active)
#pragma unroll
  for (int k = 0; k < V::NS; ++k) {
    const uint32_t d = (uint32_t)(gl + k * W);
    double tgt = 0.0, cut = 0.0;  // targetAmp reset (:1203-1208); cut 0: not targeted
#pragma unroll
    for (int c = 0; c < V::NC; ++c) {
      const uint32_t dn = t[c].up < (uint32_t)(NPM - 1) ? t[c].up + 1 : (uint32_t)DIP_LIPS;
      const bool hu = t[c].on && t[c].up == d, hd = t[c].on && dn == d;
      tgt = hu ? t[c].tup : tgt;
      cut = hu ? t[c].fc : cut;
      tgt = hd ? t[c].tdn : tgt;
      cut = hd ? t[c].fc : cut;
    }
    R.dcut[k] = cut != 0.0 ? cut : R.dcut[k];  // targeted this step: cutoff (re)assigned
    const double old = R.damp[k];
    const double amp = old + C.h.noise_amp_F * (tgt - old);
    R.damp[k] = amp;
    R.dout[k] = (old >= THR && amp < THR) ? 0.0 : R.dout[k];
    R.racc[k] = 0u;
  }
}

// One block of the rand() stream: RNG_BLOCK = 3 RJ values at ring index head, the next 10 of
// each residue chain c (i = head + 3j + c): r_{head+3j+c} = r_{head+c-3} + sum_{t<=j}
// r_{head+3t+c-31}, an inclusive prefix sum over the lanes j = 0..9 of history values, then the
// prefix sums of the outputs in sequence order.  gen == false (per utterance): everything is
// evaluated and the stores go to the sink.  The caller advances head.
template <int W, class Xc>
AFS_HD inline void rng_block(Xc &x, uint32_t *g, uint32_t *sink, int head, bool gen) {
  constexpr int RJ = rng_lanes<W>();
  const uint32_t b0 = g[RNG_R + ((head - 3) & (RNG_RING - 1))], b1 = g[RNG_R + ((head - 2) & (RNG_RING - 1))],
                 b2 = g[RNG_R + ((head - 1) & (RNG_RING - 1))], sb = g[RNG_S + ((head - 1) & (RNG_SRING - 1))];
  x.template scan_add<3>(
      [&](int gl, Lane<W> &R) {
        (void)R;
        // (every lane loads; lanes past RJ only feed their own, discarded, prefix sums)
        U4 v{{0u, 0u, 0u, 0u}};
        for (int c = 0; c < 3; ++c) v.v[c] = g[RNG_R + ((head + 3 * gl + c - 31) & (RNG_RING - 1))];
        return v;
      },
      [&](int gl, Lane<W> &R, const U4 &p) {
        const bool on = gen && gl < RJ;  // the others store into the sink
        const uint32_t n0 = b0 + p.v[0], n1 = b1 + p.v[1], n2 = b2 + p.v[2];
        *(on ? &g[RNG_R + ((head + 3 * gl) & (RNG_RING - 1))] : sink) = n0;
        *(on ? &g[RNG_R + ((head + 3 * gl + 1) & (RNG_RING - 1))] : sink) = n1;
        *(on ? &g[RNG_R + ((head + 3 * gl + 2) & (RNG_RING - 1))] : sink) = n2;
        R.rtmp[0] = n0 >> 1; R.rtmp[1] = n1 >> 1; R.rtmp[2] = n2 >> 1;
      });
  x.template scan_add<1>(
      [&](int gl, Lane<W> &R) {
        (void)gl;
        U4 v{{0u, 0u, 0u, 0u}};
        v.v[0] = R.rtmp[0] + R.rtmp[1] + R.rtmp[2];
        return v;
      },
      [&](int gl, Lane<W> &R, const U4 &p) {
        const bool on = gen && gl < RJ;
        const uint32_t s2 = sb + p.v[0], s1 = s2 - R.rtmp[2], s0 = s1 - R.rtmp[1];
        *(on ? &g[RNG_S + ((head + 3 * gl) & (RNG_SRING - 1))] : sink) = s0;
        *(on ? &g[RNG_S + ((head + 3 * gl + 1) & (RNG_SRING - 1))] : sink) = s1;
        *(on ? &g[RNG_S + ((head + 3 * gl + 2) & (RNG_SRING - 1))] : sink) = s2;
      });
}

// Phase N: noise sources (TdsModel.cpp:1630-1708), after phase_targets smoothed the
// amplitudes: the rand() draws: source d, the q-th active one in source order, takes
// draws 12q .. 12q+11 of this sample; the lanes generate the stream 30 values at a time
// (lane scans instead of one draw after another) and each source's sum of 12 draws is a
// difference of two output prefix sums.  Then the one-pole shaping filter of the owned
// active dipoles.  The values come from the ones generated ahead (rng_ahead, at least
// RNG_BLOCK pending); a sample that needs more generates further blocks here.
template <int W, int NZ, class Xc>
AFS_HD inline void phase_noise(Xc &x, double *X, const Uni &U, const Consts &C) {
  using V = NoiseV<W, NZ>;
  x.mark(PH_N_AMP);
  uint64_t act = 0;
#pragma unroll
  for (int k = 0; k < V::NS; ++k)
    act |= x.ballot([&](int gl, Lane<W> &R) { return gl + k * W < NDIP && !(R.damp[k] < THR); }) << (k * W);
  if (act == 0) {
    x.par([&](int gl, Lane<W> &R) {
      (void)R;
#pragma unroll
      for (int k = 0; k < V::NS; ++k)
        if (gl + k * W < NDIP) X[X_SMP + gl + k * W] = 0.0;
    });
    return;
  }
  uint32_t *g = (uint32_t *)(X + X_RNG);
  const int head0 = x.first().rhead, pend = x.first().rpend;
  const int base = head0 - pend;  // ring index of this sample's first draw
  const int need = 12 * __builtin_popcountll(act);
  // draws [lo, hi) of this sample are generated: add their share to the owners' sums
  // (branch-free: every slot loads its two prefix sums, inactive ones add zero)
  auto consume = [&](int lo, int hi) {
    x.par([&](int gl, Lane<W> &R) {
#pragma unroll
      for (int k = 0; k < V::NS; ++k) {
        const int d = gl + k * W;  // < 64
        const bool on = d < NDIP && ((act >> d) & 1);
        const int q0 = 12 * __builtin_popcountll(act & ((1ull << d) - 1));
        const int a = q0 > lo ? q0 : lo, b = q0 + 12 < hi ? q0 + 12 : hi;
        const uint32_t sb = g[RNG_S + ((base + b - 1) & (RNG_SRING - 1))];
        const uint32_t sa = g[RNG_S + ((base + a - 1) & (RNG_SRING - 1))];
        R.racc[k] += (on && a < b) ? sb - sa : 0u;
      }
    });
  };
  int avail = pend;
  int head = head0;
  consume(0, avail);  // (the pending values are consumed before a block here overwrites them)
  constexpr int RNG_BLOCK = 3 * rng_lanes<W>();
  while (avail < need) {  // (three or more active sources, or nothing pending yet)
    rng_block<W>(x, g, (uint32_t *)(X + X_ACT + 8), head, true);
    x.sync();
    consume(avail, avail + RNG_BLOCK);
    avail += RNG_BLOCK;
    head = (head + RNG_BLOCK) & (RNG_SRING - 1);
  }
  x.sync();
  x.mark(PH_N_RNG);
  // (every lane stores the same ring head / pending count; the shaping filter is branch-free
  // over the slots except for the exponential of a cutoff other than the clamped 2000 Hz)
  const uint64_t ndraw = *(const uint64_t *)(X + X_NDRAW) + (uint64_t)need;
  x.par([&](int gl, Lane<W> &R) {
    (void)gl; (void)R;
    R.rhead = head;
    R.rpend = avail - need;
    *(uint64_t *)(X + X_NDRAW) = ndraw;  // (every lane stores the same count)
  });
  x.par([&](int gl, Lane<W> &R) {
#pragma unroll
    for (int k = 0; k < V::NS; ++k) {
      const int d = gl + k * W;
      const bool on = d < NDIP && ((act >> d) & 1);
      double xi = (double)(int32_t)R.racc[k];
      xi *= 1.0 / 2147483647.0;  // constant reciprocals (within 1 ulp of the divisions)
      xi -= 6.0;
      xi *= 0.28867513459481288225;  // 1 / sqrt(12)
      const double cut = R.dcut[k];
      double xx = C.h.noise_x_2000;
      if (on && cut != 2000.0) xx = exp(-2.0 * PI * (cut * C.h.dt));
      double y = (1.0 - xx) * xi;
      y += xx * R.dout[k];
      R.dout[k] = on ? y : R.dout[k];
      X[d < NDIP ? X_SMP + d : X_ACT + 2] = on ? y * R.damp[k] : 0.0;
    }
  });
}

// Two blocks of the stream (2 RNG_BLOCK values at head) in one pass (gen == false: evaluated,
// stored into the sink).  The second block's history terms r_{i-31} are the first block's values,
// taken from the lanes' registers instead of a store, a wave fence and a load: its chains c = 1,
// 2 sum lane j's values c = 0, 1 of the first block, its chain c = 0 lane j-1's value 2 (lane 0:
// r_{head-1}), and its bases r_{i-3} are the first block's last lane (RJ - 1).  Every history
// load precedes the stores, which overwrite values head - 64 .. head - 5 (the second block's
// history, head - 1 .. head + 28, is in registers) and prefix sums head - RNG_SRING ..
// head - RNG_SRING + 2 RNG_BLOCK - 1.
template <int W, class Xc>
AFS_HD inline void rng_block2(Xc &x, uint32_t *g, uint32_t *sink, int head, bool gen) {
  constexpr int RJ = rng_lanes<W>(), RB = 3 * RJ;
  static_assert(RJ == 10, "ten lanes per block (the 31-value lag)");
  const uint32_t b0 = g[RNG_R + ((head - 3) & (RNG_RING - 1))], b1 = g[RNG_R + ((head - 2) & (RNG_RING - 1))],
                 b2 = g[RNG_R + ((head - 1) & (RNG_RING - 1))], sb = g[RNG_S + ((head - 1) & (RNG_SRING - 1))];
  // block 1: r_{head+3j+c} = r_{head+c-3} + sum_{t<=j} r_{head+3t+c-31}
  x.template scan_add<3>(
      [&](int gl, Lane<W> &R) {
        (void)R;
        U4 v{{0u, 0u, 0u, 0u}};
        for (int c = 0; c < 3; ++c) v.v[c] = g[RNG_R + ((head + 3 * gl + c - 31) & (RNG_RING - 1))];
        return v;
      },
      [&](int, Lane<W> &R, const U4 &p) {
        R.rtmp[0] = b0 + p.v[0];
        R.rtmp[1] = b1 + p.v[1];
        R.rtmp[2] = b2 + p.v[2];
      });
  // block 2: r_{head+RB+3j+c} = r_{head+RB+c-3} + sum_{t<=j} r_{head+3t+c-1}
  x.template pull_u<-1, 1>([&](int, Lane<W> &R) { return U4{{R.rtmp[2], 0u, 0u, 0u}}; },
                           [&](int gl, Lane<W> &R, const U4 &v) { R.rtmp[3] = gl == 0 ? b2 : v.v[0]; });
  x.template scan_add<3>([&](int, Lane<W> &R) { return U4{{R.rtmp[3], R.rtmp[0], R.rtmp[1], 0u}}; },
                         [&](int, Lane<W> &R, const U4 &p) {
                           R.rtmp[3] = p.v[0];
                           R.rtmp[4] = p.v[1];
                           R.rtmp[5] = p.v[2];
                         });
  x.template bcast_u<RJ - 1, 3>([&](int, Lane<W> &R) { return U4{{R.rtmp[0], R.rtmp[1], R.rtmp[2], 0u}}; },
                                [&](int, Lane<W> &R, const U4 &v) {
                                  R.rtmp[3] += v.v[0];
                                  R.rtmp[4] += v.v[1];
                                  R.rtmp[5] += v.v[2];
                                });
  // prefix sums of the outputs r >> 1 in sequence order: both blocks' lane sums scanned together,
  // the second block based on the first's last sum (lane RJ - 1)
  x.template scan_add<2>(
      [&](int, Lane<W> &R) {
        return U4{{(R.rtmp[0] >> 1) + (R.rtmp[1] >> 1) + (R.rtmp[2] >> 1),
                   (R.rtmp[3] >> 1) + (R.rtmp[4] >> 1) + (R.rtmp[5] >> 1), 0u, 0u}};
      },
      [&](int, Lane<W> &R, const U4 &p) {
        R.rtmp[6] = p.v[0];
        R.rtmp[7] = p.v[1];
      });
  x.template bcast_u<RJ - 1, 1>(
      [&](int, Lane<W> &R) { return U4{{R.rtmp[6], 0u, 0u, 0u}}; },
      [&](int gl, Lane<W> &R, const U4 &v) {
        const bool on = gen && gl < RJ;  // the others store into the sink
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int h = head + q * RB + 3 * gl;
          const uint32_t n0 = R.rtmp[3 * q], n1 = R.rtmp[3 * q + 1], n2 = R.rtmp[3 * q + 2];
          const uint32_t s2 = sb + (q ? v.v[0] + R.rtmp[7] : R.rtmp[6]), s1 = s2 - (n2 >> 1), s0 = s1 - (n1 >> 1);
          *(on ? &g[RNG_R + (h & (RNG_RING - 1))] : sink) = n0;
          *(on ? &g[RNG_R + ((h + 1) & (RNG_RING - 1))] : sink) = n1;
          *(on ? &g[RNG_R + ((h + 2) & (RNG_RING - 1))] : sink) = n2;
          *(on ? &g[RNG_S + (h & (RNG_SRING - 1))] : sink) = s0;
          *(on ? &g[RNG_S + ((h + 1) & (RNG_SRING - 1))] : sink) = s1;
          *(on ? &g[RNG_S + ((h + 2) & (RNG_SRING - 1))] : sink) = s2;
        }
      });
}

// The rand() stream generated ahead of its use, so that the noise phase of the next sample
// finds its draws generated: AFS_RNG_AHEAD = 2: two blocks (rng_block2) whenever fewer than two
// blocks are pending (up to five active sources, 60 draws; the usual four -- the glottis source
// and a tongue constriction, two dipoles each -- draw 48); 1: one block whenever fewer than one
// is pending (one or two active sources).  A sample that needs more generates further blocks in
// the noise phase.  It depends on the ring alone, not on the acoustic state, so it runs in the
// update block after the solver, beside the update's own chains instead of on the noise
// phase's.  With fewer than AFS_RNG_AHEAD blocks pending, the values and prefix sums a
// generation overwrites (rng_block, rng_block2) are no longer needed: neither the pending ones,
// the prefix sum before the oldest of them, nor the generator's 31-value history.  Draws are
// counted when consumed (phase_noise), so the rand() call count is the reference's.
#ifndef AFS_RNG_SKIP
#define AFS_RNG_SKIP 0  // 1: a wave none of whose utterances needs the blocks skips them (a uniform branch: slower)
#endif
template <int W, class Xc>
AFS_HD inline void rng_ahead(Xc &x, double *X) {
  constexpr int RNG_BLOCK = 3 * rng_lanes<W>();
  constexpr int GEN = AFS_RNG_AHEAD >= 2 ? 2 * RNG_BLOCK : RNG_BLOCK;  // values per generation
  static_assert(GEN <= RNG_SRING - GEN, "pending values (< GEN), the prefix sum before them and a generation fit the ring");
  static_assert(GEN <= RNG_RING, "a generation fits the value ring");
  uint32_t *g = (uint32_t *)(X + X_RNG);
  const int head = x.first().rhead, pend = x.first().rpend;
  const bool gen = pend < GEN;
  if (!AFS_RNG_SKIP || x.wave_any(gen)) {
    if constexpr (AFS_RNG_AHEAD >= 2) rng_block2<W>(x, g, (uint32_t *)(X + X_RNG_SINK), head, gen);
    else rng_block<W>(x, g, (uint32_t *)(X + X_RNG_SINK), head, gen);
  }
  x.par([&](int gl, Lane<W> &R) {
    (void)gl;
    R.rhead = gen ? ((head + GEN) & (RNG_SRING - 1)) : head;
    R.rpend = gen ? pend + GEN : pend;
  });
}

// ---------------------------------------------------------------------------
// Phase M: matrix rows (TdsModel.cpp:1785-2039), written as the SPD matrix A = -M, b = -rhs.
// Owner of section s writes row s (its in-current), the edges of section s and, for
// s = 64 / 83, the two radiation rows.
// ---------------------------------------------------------------------------
AFS_HD inline double sec_L(const double *X, const Consts &C, int s) {
  return (s >= DYN0 && s < DYN0 + NDYNS) ? X[X_L + s - DYN0] : C.stat[static_index(s)][ST_L];
}
AFS_HD inline double sec_E(const double *X, const Consts &C, int s) {
  return (s >= DYN0 && s < DYN0 + NDYNS) ? X[X_E + s - DYN0] : C.stat[static_index(s)][ST_E];
}
AFS_HD inline double sec_R1(const double *X, const Consts &C, int s) {
  return (s >= DYN0 && s < DYN0 + NDYNS) ? X[X_R1 + s - DYN0] : C.stat[static_index(s)][ST_R];
}

// The section records of this lane's slots (absent slots read the record of index NS).
template <int W>
AFS_HD inline void load_sec_recs(int gl, const Consts &C, SecRec *rec) {
#pragma unroll
  for (int j = 0; j < Shape<W>::NSL; ++j) {
    const int s = slot_section<W>(j, gl);
    rec[j] = C.sec[s < 0 ? NS : s];
  }
}

template <int W, int ROLE = ROLE_ALL>
AFS_HD inline void phase_rows(int gl, Lane<W> &R, const double *__restrict__ X, double *__restrict__ Xw,
                              const Uni &U, const Consts &C) {
  // X (reads) and Xw (writes) are the same utterance block; the phase writes only the
  // solver arrays (X_DIAG, X_RHS, X_OFF), which it never reads.  The slot loop is one
  // branch-free block: one row form serves simple and bifurcation rows, an absent slot
  // writes into the sink slots; the radiation rows follow.
  using S = Shape<W>;
  const double idt = C.h.inv_dtTH;
  const afs_options &opt = U.opt;
  SecRec rec[S::NSL];
  load_sec_recs<W>(gl, C, rec);
  Xw[X_OFF + EDGE_ZERO] = 0.0;  // the solver's zero edge (union slot; every lane stores it)
  Xw[X_DIAG + NC + 1] = 1.0;    // the arm solver's dummy pivot and rhs
  Xw[X_RHS + NC + 1] = 0.0;
  // the loads through the records' offsets (source section, partner flows, dipole sample),
  // every slot's before the arithmetic
  double xla[S::NSL], xra[S::NSL], xea[S::NSL], xda[S::NSL], xsx[S::NSL], xub[S::NSL], xurb[S::NSL], xrad[S::NSL];
#pragma unroll
  for (int j = 0; j < S::NSL; ++j) {
    if (!role_slot<ROLE>(j, S::ND)) continue;
    const SecRec &q = rec[j];
    // (the source's L, R1 and E sit at fixed distances in the dynamic arrays: one address)
    xla[j] = xat(X, q.x_la);
    xra[j] = xat(X, q.x_la + (X_R1 - X_L) * 8);
    xea[j] = xat(X, q.x_la + (X_E - X_L) * 8);
    xda[j] = xat(X, q.x_da);
    xsx[j] = xat(X, q.x_sx);
    xub[j] = xat(X, q.x_ub);
    xurb[j] = xat(X, q.x_urb);
    xrad[j] = j < S::ND ? xat(X, q.x_la + (X_RAD - X_L) * 8) : 0.0;
  }
#pragma unroll
  for (int j = 0; j < S::NSL; ++j) {
    if (!role_slot<ROLE>(j, S::ND)) continue;
    const bool dyn = j < S::ND;
    const int s0 = slot_section<W>(j, gl);
    const int s = s0 < 0 ? (dyn ? DYN0 : 0) : s0;
    const int i = s0 < 0 ? NODE_SINK : s;  // current i flows into section s
    const SecRec &q = rec[j];
    const double *ks = C.stat[dyn ? 0 : static_index(s)];  // (a dynamic slot has no row: row 0 stands in)
    const double LB = dyn ? X[X_L + s - DYN0] : ks[ST_L];
    const double RB = dyn ? X[X_R0 + s - DYN0] : ((s == S_FOSSA0 && !opt.piriform_fossa) ? C.h.fossa_R0 : ks[ST_R]);
    const double R1B = dyn ? X[X_R1 + s - DYN0] : ks[ST_R];
    const double EB = dyn ? X[X_E + s - DYN0] : ks[ST_E], DB = X[X_D + s];
    // source section a: a static source's constants come from the record, a dynamic one's
    // from X (the other term is an exact 0.0; no source: both are)
    const double LA = q.c_la + xla[j], RA = q.c_ra + xra[j], EA = q.c_ea + xea[j];
    const double DA = xda[j];
    const double LAB0 = LA + LB, RAB = RA + RB;
    double Sx = 0.0;
    Sx -= xsx[j];  // dipole sample (pharynx/mouth) or the lung pressure (section 0)
    const double uu = R.u[j], uur = R.ur[j];
    // the source section bifurcates: its other output is current br (else the zero slot: 0.0)
    const double uD = xub[j], uDr = xurb[j];
    // One row form for both cases: the bifurcation form (:1913-1965) with the partner's flows
    // 0.0 is the simple junction (:1966-2001), whose inductance may carry Sondhi's inner
    // length correction between pharynx/mouth sections.
    double LAB = LAB0;
    if (dyn) {
      const double jl = junction_l(xrad[j], X[X_RAD + s - DYN0]);
      const bool use = (opt.inner_length_corrections != 0) & ((q.flags & SR_JUNCTION) != 0) & ((q.flags & SR_BIF) == 0);
      LAB = use ? LAB + jl : LAB;  // (a select: no branch around the radii loads)
    }
    const double G = LAB * idt + RAB;
    const double H = -idt * (LAB * uu + LA * uD) - (TH1 / TH) * (LAB * uur + LA * uDr) + Sx;
    // The reference's row (TdsModel.cpp:1913-2001) is m = -E_B - G - E_A on the diagonal and
    // rhs = H + D_B - D_A; the SPD system stores -m and -rhs.  Written as the negated sums
    // themselves -- exactly the same values, negation being exact and rounding symmetric -- so
    // that no stored value needs a sign flip (a v_xor per value).
    Xw[X_DIAG + i] = (EB + G) + EA;   // -m   (E_A: 0.0 without a source)
    Xw[X_RHS + i] = DA - (H + DB);    // -rhs (D_A: 0.0 without a source)
    // edges of section s: (in, out0) = -E, (in, out1) = -E, (out0, out1) = E + L/(dt th) + R1
    xat(Xw, q.x_e0) = -EB;
    xat(Xw, q.x_e1) = -EB;
    xat(Xw, q.x_e2) = EB + (LB * idt + R1B);
  }
  constexpr int J64 = (S_LAST_MOUTH - DYN0) / W, J83 = S::ND + (S_LAST_NOSE - 46) / W;
#pragma unroll
  for (int j = 0; j < S::NSL; ++j) {
    if (j != J64 && j != J83) continue;  // (no other slot holds a radiation section)
    if (!role_slot<ROLE>(j, S::ND)) continue;
    if (!(rec[j].flags & SR_RADIATION)) continue;
    // radiation rows of s = 64 / 83 (TdsModel.cpp:1841-1911)
    const bool dyn = j < S::ND;
    const int s = slot_section<W>(j, gl);
    const double *ks = C.stat[dyn ? 0 : static_index(s)];
    const double LB = dyn ? X[X_L + s - DYN0] : ks[ST_L];
    const double R1B = dyn ? X[X_R1 + s - DYN0] : ks[ST_R];
    const double EB = dyn ? X[X_E + s - DYN0] : ks[ST_E], DB = X[X_D + s];
    const SecRec &q = rec[j];
    const int rc = q.x_rad[0] / 8 - X_U, lc = q.x_rad[1] / 8 - X_U;
    double uR = xat(X, q.x_rad[0]), uL = xat(X, q.x_rad[1]), uRr = xat(X, q.x_rad[2]), uLr = xat(X, q.x_rad[3]);
    R.rad_u[0] = uR; R.rad_u[1] = uL;
    const double LA2 = LB, RA2 = R1B, Sr = -X[X_SMP + DIP_LIPS];
    {
      const double Rrad = dyn ? X[X_RRAD] : C.h.rrad_nose;  // (network phase / tables)
      double F = LA2 * idt + RA2 + Rrad;
      double H = -(LA2 * idt) * (uR + uL) - (LA2 * (TH1 / TH)) * (uRr + uLr) + Sr;
      Xw[X_DIAG + rc] = EB + F;   // (negated sums, as the slot rows)
      Xw[X_RHS + rc] = DB - H;
    }
    {
      const double Lrad = dyn ? X[X_RRAD + 1] : C.h.lrad_nose;
      double LAB2 = LA2 + Lrad;
      double G = LAB2 * idt + RA2;
      double H = -idt * (LA2 * uR + LAB2 * uL) - (TH1 / TH) * (LA2 * uRr + LAB2 * uLr) + Sr;
      Xw[X_DIAG + lc] = EB + G;
      Xw[X_RHS + lc] = DB - H;
    }
  }
}

// ---------------------------------------------------------------------------
// Arm solver (afs_model.h ArmRec; partition and checks in afs_tables.cpp arm_records).
// The LDL^T of the per-sample matrix (the reference factors the same matrix by an envelope
// Cholesky, TdsModel.cpp:2231-2314), in an order that keeps the eliminations in registers: every lane folds the leaves of its segment and walks the segment
// from the far end (each step eliminates one node whose neighbours are the next position and
// the anchor, the previous lane's boundary, through the fill edge F), the boundaries of an arm
// are then reduced lane to lane toward the junction by DPP row shifts, the junction lane
// solves the triangle, and the solutions travel back the same way.  LDS is touched only to
// load the rows' values and to keep the walk's factors for the back substitution.
// ---------------------------------------------------------------------------
// (A negative pivot -- the reference's Cholesky takes the square root of it -- is not
// checked on the elimination chain: every lane keeps whether a pivot it met was negative, and
// after the forward pass a ballot over the utterance's lanes makes every solution NaN.)

// Phase A of a lane: the fold leaves, then the walk from the far end to the boundary.  Every
// load comes before the first store, so that the loads issue back to back (the stores go to
// LDS slots the compiler cannot tell apart from the loaded ones).
AFS_HD inline void arm_walk(const ArmRec &rr, double *X, ArmCarry &a) {
  const ArmRec r = rr;
  double D[ARM_P], Y[ARM_P], E[ARM_P - 1];
  double dl[ARM_FOLDS], yl[ARM_FOLDS], l0[ARM_FOLDS], l1[ARM_FOLDS];
#pragma unroll
  for (int p = 0; p < ARM_P; ++p) {
    D[p] = xat(X, r.d[p]);
    Y[p] = xat(X, r.d[p] + RHS_DELTA);
  }
#pragma unroll
  for (int p = 0; p < ARM_P - 1; ++p) E[p] = xat(X, r.e[p]);
#pragma unroll
  for (int f = 0; f < ARM_FOLDS; ++f) {
    dl[f] = xat(X, r.ld[f]);
    yl[f] = xat(X, r.ld[f] + RHS_DELTA);
    l0[f] = xat(X, r.le0[f]);
    l1[f] = xat(X, r.le1[f]);
  }
  const double ea = xat(X, r.ea);
  a.e28 = xat(X, r.fx0);
  a.e29 = xat(X, r.fx1);
  a.ej = xat(X, r.ej);
  const bool in = (r.flags & ARM_IN) != 0, end = (r.flags & ARM_END) != 0;
  a.sf = in ? (int)r.idx : -1;
  a.sb = (in && !end) ? (int)r.idx : -1;
  a.end = end ? 1 : 0;
  // fold slot f: the leaf joined to positions p, p+1 (an unused slot: pivot 1, zero edges)
  double il[ARM_FOLDS];
  bool neg = false;  // (lane masks: one compare per pivot, no select)
#pragma unroll
  for (int f = 0; f < ARM_FOLDS; ++f) {
    const int p = arm_fold_pos(f);
    il[f] = pivot_recip(dl[f]);
    neg = neg | (dl[f] < 0.0);
    const double f0 = l0[f] * il[f], f1 = l1[f] * il[f];
    D[p] = fma(-f0, l0[f], D[p]);
    Y[p] = fma(-f0, yl[f], Y[p]);
    D[p + 1] = fma(-f1, l1[f], D[p + 1]);
    Y[p + 1] = fma(-f1, yl[f], Y[p + 1]);
    E[p] = fma(-f0, l1[f], E[p]);
  }
  // the walk: position p has neighbours p+1 (edge E[p]) and the anchor (edge F, which the
  // anchor edge becomes at the first real position; dummy positions keep F = 0)
  double F = 0.0, dA = 0.0, yA = 0.0;
#pragma unroll
  for (int p = 0; p < ARM_P - 1; ++p) {
    if (p <= ARM_START_MAX) F = (p == (int)r.start) ? ea : F;  // (no segment starts later, arm_records)
    const double e2 = E[p] * E[p];       // (off the pivot chain: D[p+1] waits for inv only)
    const double inv = pivot_recip(D[p]);
    neg = neg | (D[p] < 0.0);
    const double g = F * inv, h = E[p] * inv;
    dA = fma(-g, F, dA);
    yA = fma(-g, Y[p], yA);
    D[p + 1] = fma(-e2, inv, D[p + 1]);
    Y[p + 1] = fma(-h, Y[p], Y[p + 1]);
#if AFS_WALK_PRESCALED
    // the back substitution's factors, scaled by the pivot's reciprocal here (g and h are needed
    // anyway): x_p = Y_p / d_p - (F_p / d_p) xA - (E_p / d_p) x_{p+1} (arm_back)
    xat(X, r.d[p] + RHS_DELTA) = Y[p] * inv;
    xat(X, r.u[p]) = g;
    xat(X, r.e[p]) = h;
#else
    xat(X, r.d[p]) = inv;                // factors for the back substitution
    xat(X, r.d[p] + RHS_DELTA) = Y[p];
    xat(X, r.u[p]) = F;
    xat(X, r.e[p]) = E[p];
#endif
    F = -(g * E[p]);                     // fill edge anchor - p+1
  }
#pragma unroll
  for (int f = 0; f < ARM_FOLDS; ++f) xat(X, r.ld[f]) = il[f];
  a.F = ((int)r.start == ARM_P - 1) ? ea : F;
  a.Db = D[ARM_P - 1];
  a.Yb = Y[ARM_P - 1];
  a.dA = dA;
  a.yA = yA;
  a.neg = neg;
}

// Back substitution of a lane's segment and leaves, from its boundary's solution a.x and the
// anchor's xA (all loads first, as in the walk); the junction lane stores the triangle's
// solutions here too (the other lanes into the sink).
AFS_HD inline void arm_back(const ArmRec &rr, const ArmJunction &J, bool junction, double *X, const ArmCarry &a,
                            double xA) {
  const ArmRec r = rr;
  double inv[ARM_P - 1], y[ARM_P - 1], Fp[ARM_P - 1], Ep[ARM_P - 1];
  double il[ARM_FOLDS], yl[ARM_FOLDS], l0[ARM_FOLDS], l1[ARM_FOLDS];
#pragma unroll
  for (int p = 0; p < ARM_P - 1; ++p) {
    inv[p] = AFS_WALK_PRESCALED ? 1.0 : xat(X, r.d[p]);  // (prescaled: Y / d, F / d, E / d)
    y[p] = xat(X, r.d[p] + RHS_DELTA);
    Fp[p] = xat(X, r.u[p]);
    Ep[p] = xat(X, r.e[p]);
  }
#pragma unroll
  for (int f = 0; f < ARM_FOLDS; ++f) {
    il[f] = xat(X, r.ld[f]);
    yl[f] = xat(X, r.ld[f] + RHS_DELTA);
    l0[f] = xat(X, r.le0[f]);
    l1[f] = xat(X, r.le1[f]);
  }
  double xs[ARM_P];
  xs[ARM_P - 1] = a.x;
#if AFS_BACK_SCALED
  // x_p = (y_p - F_p xA - E_p x_{p+1}) / d_p with the terms that do not depend on x_{p+1} scaled
  // ahead: one fma per position on the chain instead of three dependent operations
  double c[ARM_P - 1], e[ARM_P - 1];
#pragma unroll
  for (int p = 0; p < ARM_P - 1; ++p) {
    if constexpr (AFS_WALK_PRESCALED) {
      c[p] = fma(-Fp[p], xA, y[p]);
      e[p] = -Ep[p];
    } else {
      c[p] = fma(-Fp[p], xA, y[p]) * inv[p];
      e[p] = -Ep[p] * inv[p];
    }
  }
#pragma unroll
  for (int p = ARM_P - 2; p >= 0; --p) xs[p] = fma(e[p], xs[p + 1], c[p]);
#else
#pragma unroll
  for (int p = ARM_P - 2; p >= 0; --p) {
    xs[p] = fma(-Fp[p], xA, fma(-Ep[p], xs[p + 1], y[p])) * inv[p];
  }
#endif
#pragma unroll
  for (int p = 0; p < ARM_P; ++p) xat(X, r.u[p]) = xs[p];
#pragma unroll
  for (int f = 0; f < ARM_FOLDS; ++f) {
    const int p = arm_fold_pos(f);
    xat(X, r.lu[f]) = fma(-l1[f], xs[p + 1], fma(-l0[f], xs[p], yl[f])) * il[f];
  }
  const uint32_t sink = (uint32_t)(X_U + U_SINK) * 8u;
  xat(X, junction ? J.u[0] : sink) = a.xj[0];
  xat(X, junction ? J.u[1] : sink) = a.xj[1];
  xat(X, junction ? J.u[2] : sink) = a.xj[2];
}

// The same walk and back substitution with the loads issued two positions ahead instead of all
// ahead (wave pairs, sample_step_pair: the pair's kernel must fit 256 registers).  The record's
// offsets come into registers first (no LDS round trip for an address on the chain), and every
// value is computed by the same operations in the same order as arm_walk / arm_back: a fold's terms
// on positions q, q + 1 (its part on q -- pivot, rhs and the edge q - q+1 -- before the walk's step
// q - 1 updates position q, its part on q + 1 before step q), so the factors and solutions are
// bitwise theirs.  (A value loaded ahead of an earlier position's store is one that store cannot
// change: the stores go to the lane's own slots, or as constants into the shared dummy slots --
// arm_walk loads everything before any store.)
struct ArmRaw {  // position q's pivot, rhs, edge q - q+1; the fold at q's pivot, rhs, edges
  double D, Y, E, dl, yl, l0, l1;
};
AFS_HD constexpr int arm_fold_at(int q) { return q == 2 ? 0 : q == 3 ? 1 : q == 5 ? 2 : q == 6 ? 3 : -1; }
static_assert(ARM_FOLDS == 4, "fold positions 2, 3, 5, 6 (arm_fold_pos)");
AFS_HD inline ArmRaw arm_raw(const ArmRec &r, const double *X, int q) {
  ArmRaw v{0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  if (q >= ARM_P) return v;
  v.D = xat(X, r.d[q]);
  v.Y = xat(X, r.d[q] + RHS_DELTA);
  v.E = q < ARM_P - 1 ? xat(X, r.e[q]) : 0.0;
  const int f = arm_fold_at(q);
  if (f >= 0) {
    v.dl = xat(X, r.ld[f]);
    v.yl = xat(X, r.ld[f] + RHS_DELTA);
    v.l0 = xat(X, r.le0[f]);
    v.l1 = xat(X, r.le1[f]);
  }
  return v;
}
#ifndef AFS_ARM_AHEAD
#define AFS_ARM_AHEAD 1  // positions the lean walk / back substitution load ahead (1 or 2: -2 %, r06_pair_ab.txt)
#endif
AFS_HD inline void arm_walk_lean(const ArmRec &rr, double *X, ArmCarry &a) {
  const ArmRec r = rr;
  bool neg = false;
  double il[ARM_FOLDS], f1v[ARM_FOLDS], ylv[ARM_FOLDS], l1v[ARM_FOLDS];
  const double ea = xat(X, r.ea);
  a.e28 = xat(X, r.fx0);
  a.e29 = xat(X, r.fx1);
  a.ej = xat(X, r.ej);
  ArmRaw c = arm_raw(r, X, 0), n1 = AFS_ARM_AHEAD >= 2 ? arm_raw(r, X, 1) : ArmRaw{};
  double Dc = c.D, Yc = c.Y, Ec = c.E;
  double F = 0.0, dA = 0.0, yA = 0.0;
#pragma unroll
  for (int p = 0; p < ARM_P - 1; ++p) {
    if (AFS_ARM_AHEAD < 2) n1 = arm_raw(r, X, p + 1);
    const ArmRaw n2 = AFS_ARM_AHEAD >= 2 ? arm_raw(r, X, p + 2) : ArmRaw{};
    double Dn = n1.D, Yn = n1.Y, En = n1.E;
    const int fp = arm_fold_at(p), fn = arm_fold_at(p + 1);
    if (fp >= 0) {  // the fold at p: its part on p + 1
      Dn = fma(-f1v[fp], l1v[fp], Dn);
      Yn = fma(-f1v[fp], ylv[fp], Yn);
    }
    if (fn >= 0) {  // the fold at p + 1: its part on p + 1
      il[fn] = pivot_recip(n1.dl);
      neg = neg | (n1.dl < 0.0);
      const double f0 = n1.l0 * il[fn];
      f1v[fn] = n1.l1 * il[fn];
      ylv[fn] = n1.yl;
      l1v[fn] = n1.l1;
      Dn = fma(-f0, n1.l0, Dn);
      Yn = fma(-f0, n1.yl, Yn);
      En = fma(-f0, n1.l1, En);
    }
    if (p <= ARM_START_MAX) F = (p == (int)r.start) ? ea : F;
    const double e2 = Ec * Ec;
    const double inv = pivot_recip(Dc);
    neg = neg | (Dc < 0.0);
    const double g = F * inv, h = Ec * inv;
    dA = fma(-g, F, dA);
    yA = fma(-g, Yc, yA);
    Dn = fma(-e2, inv, Dn);
    Yn = fma(-h, Yc, Yn);
    xat(X, r.d[p] + RHS_DELTA) = Yc * inv;
    xat(X, r.u[p]) = g;
    xat(X, r.e[p]) = h;
    F = -(g * Ec);
    Dc = Dn;
    Yc = Yn;
    Ec = En;
    n1 = n2;
  }
#pragma unroll
  for (int f = 0; f < ARM_FOLDS; ++f) xat(X, r.ld[f]) = il[f];
  const bool in = (r.flags & ARM_IN) != 0, end = (r.flags & ARM_END) != 0;
  a.sf = in ? (int)r.idx : -1;
  a.sb = (in && !end) ? (int)r.idx : -1;
  a.end = end ? 1 : 0;
  a.F = ((int)r.start == ARM_P - 1) ? ea : F;
  a.Db = Dc;
  a.Yb = Yc;
  a.dA = dA;
  a.yA = yA;
  a.neg = neg;
}

struct ArmRawB {  // position p's rhs, fill edge, edge p - p+1; the fold at p's pivot reciprocal, rhs, edges
  double y, Fp, Ep, il, yl, l0, l1;
};
AFS_HD inline ArmRawB arm_raw_back(const ArmRec &r, const double *X, int p) {
  ArmRawB v{0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  if (p < 0) return v;
  v.y = xat(X, r.d[p] + RHS_DELTA);
  v.Fp = xat(X, r.u[p]);
  v.Ep = xat(X, r.e[p]);
  const int f = arm_fold_at(p);
  if (f >= 0) {
    v.il = xat(X, r.ld[f]);
    v.yl = xat(X, r.ld[f] + RHS_DELTA);
    v.l0 = xat(X, r.le0[f]);
    v.l1 = xat(X, r.le1[f]);
  }
  return v;
}
AFS_HD inline void arm_back_lean(const ArmRec &rr, const ArmJunction &J, bool junction, double *X, const ArmCarry &a,
                                 double xA) {
  static_assert(AFS_WALK_PRESCALED && AFS_BACK_SCALED, "the lean back substitution is the prescaled, scaled form");
  const ArmRec r = rr;
  double xn = a.x;  // x_{p+1}
  ArmRawB q1 = arm_raw_back(r, X, ARM_P - 2), q2 = AFS_ARM_AHEAD >= 2 ? arm_raw_back(r, X, ARM_P - 3) : ArmRawB{};
  xat(X, r.u[ARM_P - 1]) = xn;
#pragma unroll
  for (int p = ARM_P - 2; p >= 0; --p) {
    const ArmRawB q3 = AFS_ARM_AHEAD >= 2 ? arm_raw_back(r, X, p - 2) : arm_raw_back(r, X, p - 1);
    const double c = fma(-q1.Fp, xA, q1.y), e = -q1.Ep;
    const double xp = fma(e, xn, c);
    xat(X, r.u[p]) = xp;
    const int f = arm_fold_at(p);
    if (f >= 0) xat(X, r.lu[f]) = fma(-q1.l1, xn, fma(-q1.l0, xp, q1.yl)) * q1.il;
    xn = xp;
    if (AFS_ARM_AHEAD >= 2) {
      q1 = q2;
      q2 = q3;
    } else {
      q1 = q3;
    }
  }
  const uint32_t sink = (uint32_t)(X_U + U_SINK) * 8u;
  xat(X, junction ? J.u[0] : sink) = a.xj[0];
  xat(X, junction ? J.u[1] : sink) = a.xj[1];
  xat(X, junction ? J.u[2] : sink) = a.xj[2];
}

template <int W, class Xc, bool LEAN = false>
AFS_HD inline void solve_arms(Xc &x, double *X, const Consts &C) {
  static_assert(TREE_CHAINS == 16, "the arm partition has 16 lanes (one DPP row)");
  if constexpr (LEAN) x.lanes(TREE_CHAINS, [&](int k, Lane<W> &R) { arm_walk_lean(C.arm[k], X, R.ac); });
  else x.lanes(TREE_CHAINS, [&](int k, Lane<W> &R) { arm_walk(C.arm[k], X, R.ac); });
  // the junction triangle's values (every lane loads them; only the junction lane's matter)
  x.lanes(TREE_CHAINS, [&](int, Lane<W> &R) {
    const ArmJunction &J = C.armj;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      R.ac.jd[q] = xat(X, J.d[q]);
      R.ac.jy[q] = xat(X, J.d[q] + RHS_DELTA);
      R.ac.je[q] = xat(X, J.e[q]);
    }
    R.ac.xJ = 0.0;
  });
  // (the fossa lane's pivot reciprocal for its fold below: its boundary takes no anchor update --
  // the junction lane sends zeros -- so it is taken before the anchors' updates, off their chain)
  x.lanes(TREE_CHAINS, [&](int, Lane<W> &R) { R.ac.inv = pivot_recip(R.ac.Db); });
  // the anchors' updates: lane k's anchor is lane k-1's boundary (a first lane of an arm, the
  // fossa and the junction lane send zeros)
  x.template pull<1, 2>([&](int, Lane<W> &R) { return D4{{R.ac.dA, R.ac.yA, 0.0, 0.0}}; },
                        [&](int, Lane<W> &R, const D4 &v) { R.ac.Db += v.v[0]; R.ac.Yb += v.v[1]; });
  // the fossa lane folds 84 into 28 (lane ARM_L28) and 29 (lane ARM_L28 + 1); every other
  // lane's fossa edges are zero, so it sends zeros
  x.template pull<ARM_FOSSA - ARM_L28, 2>(
      [&](int, Lane<W> &R) {
        const double c0 = R.ac.e28 * R.ac.inv;
        return D4{{c0 * R.ac.e28, c0 * R.ac.Yb, 0.0, 0.0}};
      },
      [&](int, Lane<W> &R, const D4 &v) { R.ac.Db -= v.v[0]; R.ac.Yb -= v.v[1]; });
  x.template pull<ARM_FOSSA - ARM_L28 - 1, 3>(
      [&](int, Lane<W> &R) {
        const double c0 = R.ac.e28 * R.ac.inv, c1 = R.ac.e29 * R.ac.inv;
        return D4{{c1 * R.ac.e29, c1 * R.ac.Yb, c0 * R.ac.e29, 0.0}};
      },
      [&](int, Lane<W> &R, const D4 &v) { R.ac.Db -= v.v[0]; R.ac.Yb -= v.v[1]; R.ac.F -= v.v[2]; });
  x.lanes(TREE_CHAINS, [&](int, Lane<W> &R) { R.ac.neg = R.ac.neg | (R.ac.Db < 0.0); });
#if AFS_ARM_SCAN
  // Arm reduction toward the junction as prefix scans over the lanes (three DPP steps each
  // instead of ARM_MAXLEN - 1 dependent ones).  The boundary pivots follow d_k = D_k - F_k^2 /
  // d_{k-1} (F_k: the lane's edge to the previous lane's boundary, 0 at an arm's first lane),
  // i.e. (n_k, m_k) = M_k (n_{k-1}, m_{k-1}), M_k = [[D_k, -F_k^2], [1, 0]], d_k = n_k / m_k: the
  // lanes scan the products of their M (an arm's first lane makes the ratio independent of the
  // lanes before it); then the rhs y'_k = Yb_k - F_k y'_{k-1} / d_{k-1}, an affine recurrence.
  static_assert(ARM_MAXLEN <= 8, "three doubling steps cover an arm");
  x.lanes(TREE_CHAINS, [&](int, Lane<W> &R) {
    const double Fe = R.ac.sf >= 1 ? R.ac.F : 0.0;
    R.ac.sm[0] = R.ac.Db;
    R.ac.sm[1] = -(Fe * Fe);
    R.ac.sm[2] = 1.0;
    R.ac.sm[3] = 0.0;
  });
  // S_k <- S_k S_{k-s} (lanes before the row: the identity)
  auto mob = [&](auto sh, bool full) {
    constexpr int S_ = decltype(sh)::value;
    x.template pull<-S_, 4>([&](int, Lane<W> &R) { return D4{{R.ac.sm[0], R.ac.sm[1], R.ac.sm[2], R.ac.sm[3]}}; },
                            [&](int k, Lane<W> &R, const D4 &t) {
                              const bool in = (k & 15) >= S_;
                              const double t00 = in ? t.v[0] : 1.0, t01 = t.v[1], t10 = t.v[2], t11 = in ? t.v[3] : 1.0;
                              const double *m = R.ac.sm;
                              const double n00 = fma(m[0], t00, m[1] * t10), n10 = fma(m[2], t00, m[3] * t10);
                              if (full) {
                                const double n01 = fma(m[0], t01, m[1] * t11), n11 = fma(m[2], t01, m[3] * t11);
                                R.ac.sm[1] = n01;
                                R.ac.sm[3] = n11;
                              }
                              R.ac.sm[0] = n00;
                              R.ac.sm[2] = n10;
                            });
  };
  mob(std::integral_constant<int, 1>{}, true);
  mob(std::integral_constant<int, 2>{}, true);
  mob(std::integral_constant<int, 4>{}, false);
  x.lanes(TREE_CHAINS, [&](int, Lane<W> &R) {
    R.ac.inv = R.ac.sm[2] * pivot_recip(R.ac.sm[0]);  // 1 / d_k = m_k / n_k
    R.ac.neg = R.ac.neg | (R.ac.inv < 0.0);
  });
  x.template pull<-1, 1>([&](int, Lane<W> &R) { return D4{{R.ac.inv, 0.0, 0.0, 0.0}}; },
                         [&](int, Lane<W> &R, const D4 &v) {
                           R.ac.sm[0] = (R.ac.sf >= 1 ? -R.ac.F : 0.0) * v.v[0];
                           R.ac.sm[1] = R.ac.Yb;
                         });
  // (A, B)_k <- (A_k A_{k-s}, A_k B_{k-s} + B_k): lanes before the row read zeros, which start a chain
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    auto aff = [&](auto sh) {
      constexpr int S_ = decltype(sh)::value;
      x.template pull<-S_, 2>([&](int, Lane<W> &R) { return D4{{R.ac.sm[0], R.ac.sm[1], 0.0, 0.0}}; },
                              [&](int, Lane<W> &R, const D4 &t) {
                                R.ac.sm[1] = fma(R.ac.sm[0], t.v[1], R.ac.sm[1]);
                                R.ac.sm[0] = R.ac.sm[0] * t.v[0];
                              });
    };
    if (q == 0) aff(std::integral_constant<int, 1>{});
    if (q == 1) aff(std::integral_constant<int, 2>{});
    if (q == 2) aff(std::integral_constant<int, 4>{});
  }
  x.lanes(TREE_CHAINS, [&](int, Lane<W> &R) { R.ac.Yb = R.ac.sm[1]; });
#else
  // arm reduction toward the junction: in step s the lanes at position s of their arm
  // eliminate the previous boundary (lane k-1) from their own
  // (a lane off its step updates with a zero edge: no change, the same reciprocal again)
  x.lanes(TREE_CHAINS, [&](int, Lane<W> &R) { R.ac.inv = pivot_recip(R.ac.Db); });
#pragma unroll
  for (int s = 1; s < ARM_MAXLEN; ++s) {
    x.template pull<-1, 2>([&](int, Lane<W> &R) { return D4{{R.ac.inv, R.ac.Yb, 0.0, 0.0}}; },
                           [&](int, Lane<W> &R, const D4 &v) {
                             const double Fs = (R.ac.sf == s) ? R.ac.F : 0.0;
                             const double F2 = Fs * Fs, f = Fs * v.v[0];
                             R.ac.Db = fma(-F2, v.v[0], R.ac.Db);
                             R.ac.Yb = fma(-f, v.v[1], R.ac.Yb);
                             R.ac.inv = pivot_recip(R.ac.Db);
                           });
  }
  x.lanes(TREE_CHAINS, [&](int, Lane<W> &R) { R.ac.neg = R.ac.neg | (R.ac.Db < 0.0); });
#endif
  // the junction lane takes the three arms' last boundaries (pivot inverse, rhs, edge) and
  // solves the triangle: eliminate 65, then 41; solve 40 (uniform code on every lane)
  auto give = [&](int, Lane<W> &R) { return D4{{R.ac.inv, R.ac.Yb, R.ac.ej, 0.0}}; };
  auto take = [&](int q) {
    return [&, q](int, Lane<W> &R, const D4 &v) {
      const double g = v.v[2] * v.v[0];
      R.ac.jd[q] = fma(-g, v.v[2], R.ac.jd[q]);
      R.ac.jy[q] = fma(-g, v.v[1], R.ac.jy[q]);
    };
  };
  x.template pull<ARM_END_A - ARM_JUNCTION, 3>(give, take(0));
  x.template pull<ARM_END_B - ARM_JUNCTION, 3>(give, take(1));
  x.template pull<ARM_END_C - ARM_JUNCTION, 3>(give, take(2));
#if AFS_JUNCTION_ADJ
  // the triangle's 3 x 3 SPD system by its adjugate: cofactors, determinant and the three
  // numerators side by side, one reciprocal (9 dependent operations instead of ~16 of the
  // elimination); not positive definite (the elimination's negative pivot) <=> d2, its 2 x 2
  // minor or the determinant negative
  x.lanes(TREE_CHAINS, [&](int, Lane<W> &R) {
    const double *d = R.ac.jd, *y = R.ac.jy;
    const double e01 = R.ac.je[0], e02 = R.ac.je[1], e12 = R.ac.je[2];
    const double c00 = fma(d[1], d[2], -(e12 * e12)), c01 = fma(e02, e12, -(e01 * d[2]));
    const double c02 = fma(e01, e12, -(e02 * d[1])), c11 = fma(d[0], d[2], -(e02 * e02));
    const double c12 = fma(e01, e02, -(d[0] * e12)), c22 = fma(d[0], d[1], -(e01 * e01));
    const double det = fma(d[0], c00, fma(e01, c01, e02 * c02));
    const bool dneg = (d[2] < 0.0) | (c00 < 0.0) | (det < 0.0);
    const double r = dneg ? NAN : pivot_recip(det);
    R.ac.xj[0] = fma(c00, y[0], fma(c01, y[1], c02 * y[2])) * r;
    R.ac.xj[1] = fma(c01, y[0], fma(c11, y[1], c12 * y[2])) * r;
    R.ac.xj[2] = fma(c02, y[0], fma(c12, y[1], c22 * y[2])) * r;
  });
#else
  x.lanes(TREE_CHAINS, [&](int, Lane<W> &R) {
    double *d = R.ac.jd, *y = R.ac.jy;
    double e01 = R.ac.je[0];
    const double e02 = R.ac.je[1], e12 = R.ac.je[2];
    const double i2 = pivot_recip(d[2]);
    const double g0 = e02 * i2, g1 = e12 * i2;
    d[0] = fma(-g0, e02, d[0]);
    y[0] = fma(-g0, y[2], y[0]);
    d[1] = fma(-g1, e12, d[1]);
    y[1] = fma(-g1, y[2], y[1]);
    e01 = fma(-g0, e12, e01);
    const double i1 = pivot_recip(d[1]);
    const double h = e01 * i1;
    d[0] = fma(-h, e01, d[0]);
    y[0] = fma(-h, y[1], y[0]);
    const bool dneg = (d[0] < 0.0) | (d[1] < 0.0) | (d[2] < 0.0);
    const double x0 = dneg ? NAN : y[0] * pivot_recip(d[0]);
    const double x1 = fma(-e01, x0, y[1]) * i1;
    R.ac.xj[0] = x0;
    R.ac.xj[1] = x1;
    R.ac.xj[2] = fma(-e12, x1, fma(-e02, x0, y[2])) * i2;
  });
#endif
  x.template pull<ARM_JUNCTION - ARM_END_A, 1>([&](int, Lane<W> &R) { return D4{{R.ac.xj[0], 0.0, 0.0, 0.0}}; },
                                               [&](int k, Lane<W> &R, const D4 &v) { if (k == ARM_END_A) R.ac.xJ = v.v[0]; });
  x.template pull<ARM_JUNCTION - ARM_END_B, 1>([&](int, Lane<W> &R) { return D4{{R.ac.xj[1], 0.0, 0.0, 0.0}}; },
                                               [&](int k, Lane<W> &R, const D4 &v) { if (k == ARM_END_B) R.ac.xJ = v.v[0]; });
  x.template pull<ARM_JUNCTION - ARM_END_C, 1>([&](int, Lane<W> &R) { return D4{{R.ac.xj[2], 0.0, 0.0, 0.0}}; },
                                               [&](int k, Lane<W> &R, const D4 &v) {
                                                 R.ac.xJ = (k == ARM_END_C) ? v.v[0] : R.ac.xJ;
                                               });
  // back along the arms
  x.template pull<1, 1>([&](int, Lane<W> &R) { return D4{{R.ac.F, 0.0, 0.0, 0.0}}; },
                        [&](int, Lane<W> &R, const D4 &v) { R.ac.Fn = v.v[0]; });
#if AFS_ARM_SCAN
  // x_k = (Yb_k - Fn_k x_{k+1}) / d_k along an arm, x = (Yb - ej xJ) / d at its last lane: an
  // affine recurrence toward the arms' far ends, scanned (lanes past the row read zeros: the arms'
  // last lanes, the fossa and the junction lane have no successor term)
  x.lanes(TREE_CHAINS, [&](int, Lane<W> &R) {
    const bool mid = R.ac.sb >= 0;
    R.ac.sm[0] = mid ? -R.ac.Fn * R.ac.inv : 0.0;
    R.ac.sm[1] = mid ? R.ac.Yb * R.ac.inv : (R.ac.end ? fma(-R.ac.ej, R.ac.xJ, R.ac.Yb) * R.ac.inv : 0.0);
  });
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    auto aff = [&](auto sh) {
      constexpr int S_ = decltype(sh)::value;
      x.template pull<S_, 2>([&](int, Lane<W> &R) { return D4{{R.ac.sm[0], R.ac.sm[1], 0.0, 0.0}}; },
                             [&](int, Lane<W> &R, const D4 &t) {
                               R.ac.sm[1] = fma(R.ac.sm[0], t.v[1], R.ac.sm[1]);
                               R.ac.sm[0] = R.ac.sm[0] * t.v[0];
                             });
    };
    if (q == 0) aff(std::integral_constant<int, 1>{});
    if (q == 1) aff(std::integral_constant<int, 2>{});
    if (q == 2) aff(std::integral_constant<int, 4>{});
  }
  x.lanes(TREE_CHAINS, [&](int, Lane<W> &R) { R.ac.x = R.ac.sm[1]; });
#else
  x.lanes(TREE_CHAINS, [&](int, Lane<W> &R) {
    R.ac.x = R.ac.end ? fma(-R.ac.ej, R.ac.xJ, R.ac.Yb) * R.ac.inv : 0.0;
  });
#pragma unroll
  for (int s = ARM_MAXLEN - 2; s >= 0; --s) {
    x.template pull<1, 1>([&](int, Lane<W> &R) { return D4{{R.ac.x, 0.0, 0.0, 0.0}}; },
                          [&](int, Lane<W> &R, const D4 &v) {
                            const bool on = R.ac.sb == s;
                            R.ac.x = on ? fma(-R.ac.Fn, v.v[0], R.ac.Yb) * R.ac.inv : R.ac.x;
                          });
  }
#endif
  // the fossa lane: 84 from 28 and 29
  x.template pull<ARM_L28 - ARM_FOSSA, 1>([&](int, Lane<W> &R) { return D4{{R.ac.x, 0.0, 0.0, 0.0}}; },
                                          [&](int, Lane<W> &R, const D4 &v) { R.ac.Fn = v.v[0]; });
  x.template pull<ARM_L28 + 1 - ARM_FOSSA, 1>([&](int, Lane<W> &R) { return D4{{R.ac.x, 0.0, 0.0, 0.0}}; },
                                              [&](int k, Lane<W> &R, const D4 &v) {
                                                const double t = fma(-R.ac.e29, v.v[0], fma(-R.ac.e28, R.ac.Fn, R.ac.Yb));
                                                R.ac.x = (k == ARM_FOSSA) ? t * R.ac.inv : R.ac.x;
                                              });
  // a negative pivot anywhere: every solution of this sample is NaN (as the reference's
  // Cholesky produces from the square root of a negative pivot on)
  const bool bad = x.ballot([&](int gl, Lane<W> &R) { return gl < TREE_CHAINS && R.ac.neg; }) != 0;
  x.lanes(TREE_CHAINS, [&](int, Lane<W> &R) {
    R.ac.x = bad ? NAN : R.ac.x;
#pragma unroll
    for (int q = 0; q < 3; ++q) R.ac.xj[q] = bad ? NAN : R.ac.xj[q];
  });
  x.mark(PH_FORWARD);
  // every lane's segment from its boundary and its anchor (lane k-1's boundary)
  x.template pull<-1, 1>([&](int, Lane<W> &R) { return D4{{R.ac.x, 0.0, 0.0, 0.0}}; },
                         [&](int, Lane<W> &R, const D4 &v) { R.ac.xJ = v.v[0]; });
  if constexpr (LEAN)
    x.lanes(TREE_CHAINS, [&](int k, Lane<W> &R) { arm_back_lean(C.arm[k], C.armj, k == ARM_JUNCTION, X, R.ac, R.ac.xJ); });
  else
    x.lanes(TREE_CHAINS, [&](int k, Lane<W> &R) { arm_back(C.arm[k], C.armj, k == ARM_JUNCTION, X, R.ac, R.ac.xJ); });
  x.sync();
  x.mark(PH_BACKWARD);
}

// ---------------------------------------------------------------------------
// Phase U: updateVariables (TdsModel.cpp:2046-2098).
// ---------------------------------------------------------------------------
template <int W, int ROLE = ROLE_ALL>
AFS_HD inline void phase_update(int gl, Lane<W> &R, const double *__restrict__ X, double *__restrict__ Xw,
                                const Uni &U, const Consts &C) {
  // X (reads) and Xw (writes) are the same utterance block; the phase publishes into X_UR,
  // X_UN, X_P4, X_TVP and the sink slot, none of which it reads.  The slot loop is one
  // branch-free block (an absent slot updates a copy of section 0 and publishes into the
  // sink), so the scheduler can batch the loads of all slots; the per-section extras follow.
  using S = Shape<W>;
  const double c = C.h.noise_lp_c, idt = C.h.inv_dtTH;
  SecRec rec[S::NSL];
  load_sec_recs<W>(gl, C, rec);
  // every slot's loads first (the solution, the output flows, D and E), then the arithmetic
  double unew[S::NSL], cout[S::NSL], Ds[S::NSL], Es[S::NSL];
#pragma unroll
  for (int j = 0; j < S::NSL; ++j) {
    if (!role_slot<ROLE>(j, S::ND)) continue;
    const int s0 = slot_section<W>(j, gl);
    const int s = s0 < 0 ? (j < S::ND ? DYN0 : 0) : s0;
    unew[j] = X[X_U + s];
    cout[j] = 0.0;
    cout[j] += xat(X, rec[j].x_o0);  // 0.0 for an absent output
    cout[j] += xat(X, rec[j].x_o1);
    Ds[j] = X[X_D + s];
    Es[j] = j < S::ND ? X[X_E + s - DYN0] : C.stat[static_index(s)][ST_E];
  }
#pragma unroll
  for (int j = 0; j < S::NSL; ++j) {
    if (!role_slot<ROLE>(j, S::ND)) continue;
    const int s0 = slot_section<W>(j, gl);
    const int s = s0 < 0 ? (j < S::ND ? DYN0 : 0) : s0;
    double alpha, beta;
    if (j < S::ND) { alpha = R.al[j]; beta = R.be[j]; }
    else { alpha = C.stat[static_index(s)][ST_ALPHA]; beta = static_beta<W>(R, j, U, C, s); }  // same values as phase_network
    const double un = unew[j];
    const double uold = R.u[j];
    R.u[j] = un;
    R.ur[j] = (un - uold) * idt - (TH1 / TH) * R.ur[j];
    R.un[j] = (1.0 - c) * un + c * R.un[j];
    double cin = 0.0;
    cin += un;
    double net = cin - cout[j];
    double old = R.p[j];
    double p = Ds[j] + Es[j] * net;
    R.p[j] = p;
    double prr = (p - old) * idt - R.pr[j] * (TH1 / TH);
    R.pr[j] = prr;
    double ow = R.w[j], owr = R.wr[j];
    double w = prr * alpha + beta;
    R.w[j] = w;
    double wr = (w - ow) * idt - owr * (TH1 / TH);
    R.wr[j] = wr;
    R.wr2[j] = (wr - owr) * idt - R.wr2[j] * (TH1 / TH);
  }
  // publish (all stores after all loads: the scheduler may batch the loads of every slot)
#pragma unroll
  for (int j = 0; j < S::NSL; ++j) {
    if (!role_slot<ROLE>(j, S::ND)) continue;
    xat(Xw, rec[j].x_ur) = R.ur[j];  // for the bifurcation partner (or the sink)
    xat(Xw, rec[j].x_un) = R.un[j];  // for the noise sources (or the sink)
    xat(Xw, rec[j].x_p4) = R.p[j];   // p[22..25] for the glottis (or the sink)
  }
#pragma unroll
  for (int j = 0; j < S::NSL; ++j) {
    if (!role_slot<ROLE>(j, S::ND)) continue;
    const int s = slot_section<W>(j, gl);
    // transvelar filter inputs p[43], p[67]: only the slots that can hold sections 43 / 67
    // store, a lane without them into the sink (no branch)
    constexpr int J43 = (S_MOUTH0 + 2 - DYN0) / W, J67 = (S_NOSE0 + 2 - DYN0) / W;
    if (j == J43 || j == J67) {
      const bool tv = U.opt.transvelar_coupling != 0;
      const int dst = (tv & (s == S_MOUTH0 + 2)) ? X_TVP : (tv & (s == S_NOSE0 + 2)) ? X_TVP + 1 : X_U + U_SINK;
      Xw[dst] = R.p[j];
    }
    constexpr int J64 = (S_LAST_MOUTH - DYN0) / W, J83 = S::ND + (S_LAST_NOSE - 46) / W;
    if ((j == J64 || j == J83) && (rec[j].flags & SR_RADIATION)) {  // the two radiation currents of s = 64 / 83
      const SecRec &q = rec[j];
      for (int k = 0; k < 2; ++k) {
        double un = xat(X, q.x_rad[k]);
        // (the previous sample's d/dt and smoothed flow are still in their LDS slots: read before
        // this update overwrites them, instead of carrying them in registers through the solver:
        // +0.2 %, profiles/r03ab_ab.txt)
        const double our = xat(Xw, q.x_rad[2 + k]), oun = xat(Xw, q.x_rad[4 + k]);
        double ur = (un - R.rad_u[k]) * idt - (TH1 / TH) * our;
        xat(Xw, q.x_rad[2 + k]) = ur;
        xat(Xw, q.x_rad[4 + k]) = (1.0 - c) * un + c * oun;
      }
    }
  }
}

// The new pressure of dynamic section s from the solution, as phase_update computes it (the
// same operations on the same values), for readers in the update phase itself.
AFS_HD inline double section_pressure(const double *X, const Consts &C, int s) {
  const SecRec &q = C.sec[s];
  double cin = 0.0;
  cin += X[X_U + s];
  double cout = 0.0;
  cout += xat(X, q.x_o0);
  cout += xat(X, q.x_o1);
  const double net = cin - cout;
  return X[X_D + s] + X[X_E + s - DYN0] * net;
}

// The output stage after the radiated flow (Synthesizer.cpp:614-627): dU/dt, the 8-pole
// Chebyshev low-pass, x 0.004 / 32767.  It does not feed back into the tube, so it can run
// over a whole hop of flows afterwards (output_filter_run) or per sample (output_filter_one);
// both evaluate the same operations on the same state (X_PREVFLOW, X_OUTF).
AFS_HD inline double output_filter_one(double *X, const Consts &C, double flow) {
#pragma clang fp contract(off)
  double op = (flow - X[X_PREVFLOW]) * C.h.inv_dt;
  X[X_PREVFLOW] = flow;
  double y = iir_run<8>(X + X_OUTF, C.h.out_a, C.h.out_b, op);
  double smp = y * 0.004;
  smp = smp * (1.0 / 32767);
  if (!isfinite(smp)) X[X_NONFIN] = 1.0;
  return smp;
}

// o[0..n) holds the radiated flows of n consecutive samples; they are replaced by the audio
// samples.  The filter state stays in registers over the run.  Whole blocks of 8 samples keep the
// filters' histories in windows (x and y of the last 8 + the block's 8 samples, oldest first), so
// that sample i of a block reads its taps at fixed window positions and the window moves once per
// block (8 moves instead of 56 per block and filter); the loads of the next block are issued before
// the current one is filtered (clamped indices: no branch), and the last n % 8 samples run one by
// one.  (In K1, where the filter ran until round 3, the windows' registers pushed persistent state
// into AGPRs: -2 %, profiles/r03w_ab.txt; K6 has the registers to spare.)
// TONE: first the glottal-tone filter (skin radiation, TdsModel.cpp:687-705) over p25[i], section
// 25's new pressure of sample i, its output added to the flow o[i] (the same operations as
// phase_output, so bitwise the same audio): one loop, so that the tone chain of sample i + 1 and
// the output filter's chain of sample i (independent) overlap, instead of two runs back to back.
template <bool TONE>
AFS_HD inline void output_filter_run_t(double *X, const Consts &C, double *o, int n, const double *p25) {
  // (not contracted into fmas: each product and sum rounds as in the reference, so the result does
  // not depend on where a run starts -- a session's per-call runs equal one run over the whole
  // trajectory bit for bit; with contraction the compiler may pair the terms differently in
  // different unrolled positions)
#pragma clang fp contract(off)
  double wx[16], wy[16], ca[9], cb[9];  // wx[7 - k] = x_{t-1-k} at a block's start (wx[7]: newest)
#pragma unroll
  for (int k = 0; k < 8; ++k) { wx[7 - k] = X[X_OUTF + k]; wy[7 - k] = X[X_OUTF + 8 + k]; }
#pragma unroll
  for (int k = 0; k <= 8; ++k) { ca[k] = C.h.out_a[k]; cb[k] = C.h.out_b[k]; }
  const double inv_dt = C.h.inv_dt;
  double prev = X[X_PREVFLOW];
  bool nonfin = false;
  double tx[12], ty[12], ta[5], tb[5];  // tone filter windows: tx[3 - k] = x_{t-1-k}
  if constexpr (TONE) {
#pragma unroll
    for (int k = 0; k < 4; ++k) { tx[3 - k] = X[X_TONE + k]; ty[3 - k] = X[X_TONE + 4 + k]; }
#pragma unroll
    for (int k = 0; k <= 4; ++k) { ta[k] = C.h.tone_a[k]; tb[k] = C.h.tone_b[k]; }
  }
  // one sample with its taps at window offset b (sample i of a block: b = i)
  auto step = [&](int b, double flow, double xp) -> double {
    if constexpr (TONE) {
      double tacc = ta[0] * xp;
#pragma unroll
      for (int k = 1; k <= 4; ++k) {
        tacc += ta[k] * tx[4 + b - k];
        tacc += tb[k] * ty[4 + b - k];
      }
      tx[4 + b] = xp;
      ty[4 + b] = tacc;
      flow += tacc;
    }
    const double op = (flow - prev) * inv_dt;
    prev = flow;
    double acc = ca[0] * op;
#pragma unroll
    for (int k = 1; k <= 8; ++k) {
      acc += ca[k] * wx[8 + b - k];
      acc += cb[k] * wy[8 + b - k];
    }
    wx[8 + b] = op;
    wy[8 + b] = acc;
    double smp = acc * 0.004;
    smp = smp * (1.0 / 32767);
    nonfin = nonfin || !isfinite(smp);
    return smp;
  };
  auto shift = [&](int m) {  // the window after m samples: drop the m oldest entries
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (j + m < 16) { wx[j] = wx[j + m]; wy[j] = wy[j + m]; }
    }
    if constexpr (TONE) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j + m < 12) { tx[j] = tx[j + m]; ty[j] = ty[j + m]; }
      }
    }
  };
  const int nb = n / 8 * 8;
  double f[8], fp[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int q = i < n ? i : (n > 0 ? n - 1 : 0);
    f[i] = n > 0 ? o[q] : 0.0;
    fp[i] = (TONE && n > 0) ? p25[q] : 0.0;
  }
  for (int t0 = 0; t0 < nb; t0 += 8) {
    double g[8], gp[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // (the next block's inputs; indices clamped into the run)
      const int q = t0 + 8 + i < n ? t0 + 8 + i : n - 1;
      g[i] = o[q];
      gp[i] = TONE ? p25[q] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) o[t0 + i] = step(i, f[i], fp[i]);
    shift(8);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      f[i] = g[i];
      fp[i] = gp[i];
    }
  }
  for (int t = nb; t < n; ++t) {  // the last n % 8 samples
    o[t] = step(0, o[t], TONE ? p25[t] : 0.0);
    shift(1);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) { X[X_OUTF + k] = wx[7 - k]; X[X_OUTF + 8 + k] = wy[7 - k]; }
  X[X_PREVFLOW] = prev;
  if (nonfin) X[X_NONFIN] = 1.0;
  if constexpr (TONE) {
#pragma unroll
    for (int k = 0; k < 4; ++k) { X[X_TONE + k] = tx[3 - k]; X[X_TONE + 4 + k] = ty[3 - k]; }
  }
}

AFS_HD inline void output_filter_run(double *X, const Consts &C, double *o, int n) {
  output_filter_run_t<false>(X, C, o, n, nullptr);
}
// the glottal-tone filter and the output stage over n samples in one loop (K6 of the tone-in-K6 build)
AFS_HD inline void tone_output_run(double *X, const Consts &C, const double *p25, double *o, int n) {
  output_filter_run_t<true>(X, C, o, n, p25);
}

// Hops of at least this many samples run the output filter once per hop (output_filter_run)
// instead of inside the sample step.
constexpr int OUT_DEFER_MIN_HOP = 32;

// Phase O (lane-uniform): radiated flow and glottal tone (TdsModel.cpp:687-705); with
// defer == false also the output filter.  Returns the audio sample, or with defer the flow.
// p25 = the new pressure of section 25 (section_pressure), the glottal tone filter's input.
// The radiated flow alone (the device kernel: the glottal-tone filter runs in K6 from the
// stored p[25], tone_output_run).
AFS_HD inline double phase_output_flow(const double *X) {
  double flow = 0.0;
  flow += X[X_U + 93];
  flow += X[X_U + 94];
  flow += X[X_U + 95];
  flow += X[X_U + 96];
  return flow;
}

AFS_HD inline double phase_output(double *X, const Uni &U, const Consts &C, double p25, bool defer) {
  double flow = 0.0;
  flow += X[X_U + 93];
  flow += X[X_U + 94];
  flow += X[X_U + 95];
  flow += X[X_U + 96];
  // (the tone filter runs either way, its output is selected: no branch in the output stage)
  const double tone = iir_run<4>(X + X_TONE, C.h.tone_a, C.h.tone_b, p25);
  flow += U.opt.radiation_from_skin ? tone : 0.0;
  if (defer) return flow;
  return output_filter_one(X, C, flow);
}

// ---------------------------------------------------------------------------
// One audio sample.  Xc: execution policy (par / one / lanes / sync).
// ---------------------------------------------------------------------------

template <int W, int MODEL, bool VARLOSS, int NZ, class Xc>
AFS_HD inline double geometry_network(Xc &x, double *X, const Uni &U, const Consts &C, double ratio) {
  // the glottis of this sample: its loads first, its stores (displacements, interpolated
  // controls) at the end of the block, so that the network and the targets need not wait for
  // the glottis chain before they load
  GlotRes g{};
  x.par_uniform([&](int gl, Lane<W> &R) { phase_interpolate<W>(gl, R, X, C, ratio); },
                [&](Lane<W> &R) {
                  (void)R;
                  const double p4[4] = {X[X_P4 + 0], X[X_P4 + 1], X[X_P4 + 2], X[X_P4 + 3]};
                  if constexpr (Xc::kGlottisSplit && MODEL == AFS_GLOTTIS_TRIANGULAR)
                    g = glottis_eval_split(glottis_inputs(X), C, ratio, p4, x.half8(),
                                           [&](double v) { return x.xch8(v); });
                  else
                    g = glottis_eval<MODEL>(glottis_inputs(X), C, ratio, p4);
                });
  x.mark(PH_GEOMETRY);  // (phase marks: cycle accounting of tools/phase_prof, no-ops otherwise)
  x.dyn_neighbors();
  x.par([&](int gl, Lane<W> &R) { phase_network<W, VARLOSS>(gl, R, X, U, C, g.go); });
  x.mark(PH_NETWORK);
  // (NZ_DYN: the targets run after the block, in the variant's noise phase)
  if constexpr (NZ != NZ_DYN) x.par([&](int gl, Lane<W> &R) { phase_targets<W, NZ>(x, gl, R, X, C, g.go.a1); });
  x.par_uniform([&](int gl, Lane<W> &R) { (void)gl; (void)R; },
                [&](Lane<W> &R) { (void)R; glottis_commit(X, g); });
  return g.go.a1;
}

// The targets and noise phases of variant NZ (NZ_DYN: sample_step), after the geometry / network
// block: a phase of their own between two wave fences, so that the variants' branch splits no
// block the scheduler interleaves.
template <int W, int NZ, class Xc>
AFS_HD inline void targets_noise(Xc &x, double *X, const Uni &U, const Consts &C, double a_glot_up) {
  x.par([&](int gl, Lane<W> &R) { phase_targets<W, NZ>(x, gl, R, X, C, a_glot_up); });
  if (U.opt.generate_noise_sources) {
    phase_noise<W, NZ>(x, X, U, C);
  } else {
    x.par([&](int gl, Lane<W> &R) {
      (void)R;
      for (int d = gl; d < NDIP; d += W) X[X_SMP + d] = 0.0;
    });
  }
}

// One audio sample at `ratio` with glottis model MODEL (one kernel per model: a kernel holding
// both models' code needs more registers than the SIMD has) and noise-phase variant NZ.
// NZ = NZ_DYN: the noise-phase variant nz (wave-uniform) is chosen at run time in the phase after
// the geometry / network block (one copy of everything else); any other NZ: that variant, the
// targets inside the block.
template <int W, int MODEL, int NZ = NZ_FULL, class Xc>
AFS_HD inline void sample_step(Xc &x, double *X, const Uni &U, const Consts &C, double ratio, bool defer_out,
                               int nz = NZ_FULL) {
  static_assert(W >= TREE_CHAINS, "every solver lane needs a lane of the utterance");
  // geometry and network in one block (no LDS round trip between them): the interpolated
  // areas stay in the lanes, the neighbours' come by lane exchange, the glottis values are
  // lane-uniform
  // (one instantiation per glottis model and entrance-loss kind: no option branch in the block)
  const bool varloss = U.opt.glottis_loss == AFS_ENTRANCE_LOSS_VARIABLE;
  const double a_glot_up = varloss ? geometry_network<W, MODEL, true, NZ>(x, X, U, C, ratio)
                                   : geometry_network<W, MODEL, false, NZ>(x, X, U, C, ratio);
  x.sync();
  x.mark(PH_TARGETS);
  if constexpr (NZ == NZ_DYN) {
    (void)nz;
    // (only the variants of AFS_NZ_SET are compiled; the CPU emulator compiles them all)
    if ((AFS_NZ_SET & 2) && nz == NZ_GLOTTIS) targets_noise<W, NZ_GLOTTIS>(x, X, U, C, a_glot_up);
    else if ((AFS_NZ_SET & 1) && nz == NZ_TONGUE1) targets_noise<W, NZ_TONGUE1>(x, X, U, C, a_glot_up);
    else if ((AFS_NZ_SET & 4) && nz == NZ_T1ALL) targets_noise<W, NZ_T1ALL>(x, X, U, C, a_glot_up);
    else targets_noise<W, NZ_FULL>(x, X, U, C, a_glot_up);
  } else {
    (void)a_glot_up;
    (void)nz;
    if (U.opt.generate_noise_sources) {
      phase_noise<W, NZ>(x, X, U, C);
    } else {
      x.par([&](int gl, Lane<W> &R) {
        (void)R;
        for (int d = gl; d < NDIP; d += W) X[X_SMP + d] = 0.0;
      });
    }
  }
  x.sync();
  x.mark(PH_NOISE);
  x.par([&](int gl, Lane<W> &R) { phase_rows<W>(gl, R, X, X, U, C); });
  x.sync();
  x.mark(PH_ROWS);
  solve_arms<W>(x, X, C);
  // the rand() stream ahead of the next sample's noise phase (independent of the acoustic
  // state; here it measured best: before the rows +0.9 %, inside the solver +0.3 %)
  rng_ahead<W>(x, X);
  // the state update and the output stage (lane-uniform: radiated flow, filters) in one phase
  x.par_uniform([&](int gl, Lane<W> &R) { phase_update<W>(gl, R, X, X, U, C); },
                [&](Lane<W> &R) {
                  if constexpr (Xc::kToneOut) R.sample = phase_output_flow(X);
                  else R.sample = phase_output(X, U, C, section_pressure(X, C, S_PHARYNX0), defer_out);
                });
  x.sync();
  x.mark(PH_UPDATE);
  x.mark(PH_OUTPUT);
}


// One sample on a wave pair (tree_kernel.h, AFS_PAIR): the wave of role ROLE runs its half of the
// phases; the pair's waves meet at a workgroup barrier (x.bar()) between the four phase groups, so
// LDS carries everything one wave writes and the other reads (the dynamic slots' L, R, E, D and the
// static slots' D, the dipole samples, the rows, the solution, the published pressures and flows).
//   P1  DYN: interpolation, the glottis and its commit, [barrier], the dynamic slots' network
//       STAT: the static slots' D, [barrier], targets, noise
//       (AFS_PAIR_SPLIT1=0: no barrier inside P1, both waves evaluate the glottis, STAT commits it)
//   P2  rows of each role's slots
//   P3  STAT: the arm solver (lean form) and the rand() blocks ahead
//   P4  the state update of each role's slots; DYN: the radiated flow (R.sample)
// Both waves read the glottis displacements at the start of P1 and STAT commits the new ones in P1:
// two buffers, sample parity par reads X_RELX (par 0) or X_RELX2 and writes the other.
#if AFS_PAIR
#ifndef AFS_PAIR_LEAN
#define AFS_PAIR_LEAN 1  // the STAT wave's solver in the lean form (arm_walk_lean; 0: arm_walk, every load ahead)
#endif
#ifndef AFS_PAIR_PRIO
// the STAT wave's issue priority over its SIMD's other wave (a DYN wave of another workgroup): 1 during
// the solver, 2 during the first phase group and the solver, 3 always; 0: the launch's mode
// (TreeArgs::stat_prio, the executor's prio) -- nonzero values fix it at compile time (A/B builds)
#define AFS_PAIR_PRIO 0
#endif
template <class Xc> AFS_HD inline int pair_prio(const Xc &x) { return AFS_PAIR_PRIO ? AFS_PAIR_PRIO : x.prio; }
#ifndef AFS_PAIR_SPLIT1
// the first phase group in two: the DYN wave evaluates and commits the glottis alone (the STAT wave
// its static network meanwhile), a barrier, then DYN's network beside STAT's targets and noise (0:
// both waves evaluate the glottis, no barrier inside the group; 1 measured -2.7 %, r06_pair_ab.txt)
#define AFS_PAIR_SPLIT1 0  // (2: DYN commits the glottis, STAT evaluates its upper area alone, no barrier)
#endif
#ifndef AFS_PAIR_RNG_DYN
#define AFS_PAIR_RNG_DYN 1  // the rand() blocks ahead on the DYN wave during the solver (0: on the STAT wave after it)
#endif
template <int W, int MODEL, int NZ, int ROLE, bool VARLOSS, class Xc>
AFS_HD inline void sample_step_pair_v(Xc &x, double *X, const Uni &U, const Consts &C, double ratio, int par) {
  static_assert(ROLE == ROLE_DYN || ROLE == ROLE_STAT, "a wave pair's roles");
// (scheduling barriers between the phase groups: the scheduler otherwise mixes their code and keeps
// values of both live at once -- the pair kernel must fit 256 registers; with AFS_PAIR_MARKS named
// markers in the assembly instead, for spill accounting)
#if defined(AFS_PAIR_MARKS) && defined(__HIP_DEVICE_COMPILE__)
#define AFS_PM(t) __asm__ volatile(t)
#else
#define AFS_PM(t) AFS_SCHED_BARRIER()
#endif
  AFS_PM(";MARK P1 begin");
  if constexpr (ROLE == ROLE_STAT) {
    if (pair_prio(x) == 2) AFS_SETPRIO(2);
  }
  const int rcur = par ? X_RELX2 : X_RELX, rnext = par ? X_RELX : X_RELX2;
  // (SPLIT1 2: DYN commits the glottis, STAT evaluates only the upper area it needs -- the
  // triangular model's split form; the two-mass model keeps both evaluations)
  constexpr bool kSplitA = AFS_PAIR_SPLIT1 == 2 && MODEL == AFS_GLOTTIS_TRIANGULAR && Xc::kGlottisSplit;
  constexpr bool kDynCommit = AFS_PAIR_SPLIT1 == 1 || kSplitA;
  if constexpr (ROLE == ROLE_DYN) {
    GlotRes g{};
    x.par_uniform([&](int gl, Lane<W> &R) { phase_interpolate<W>(gl, R, X, C, ratio); },
                  [&](Lane<W> &R) {
                    (void)R;
                    const double p4[4] = {X[X_P4 + 0], X[X_P4 + 1], X[X_P4 + 2], X[X_P4 + 3]};
                    if constexpr (Xc::kGlottisSplit && MODEL == AFS_GLOTTIS_TRIANGULAR)
                      g = glottis_eval_split(glottis_inputs(X, rcur), C, ratio, p4, x.half8(),
                                             [&](double v) { return x.xch8(v); });
                    else
                      g = glottis_eval<MODEL>(glottis_inputs(X, rcur), C, ratio, p4);
                    if constexpr (kDynCommit) glottis_commit(X, g, rnext);
                    if constexpr (AFS_PAIR_SPLIT1 == 1) X[X_AGLOT] = g.go.a1;
                  });
    x.mark(PH_D_GEO);
    if constexpr (AFS_PAIR_SPLIT1 == 1) {
      x.bar();
      x.mark(PH_P0WAIT);
    }
    x.dyn_neighbors();
    x.par([&](int gl, Lane<W> &R) { phase_network<W, VARLOSS, ROLE_DYN>(gl, R, X, U, C, g.go); });
    x.mark(PH_NETWORK);
  } else {
    double a_glot_up = 0.0;
    if constexpr (AFS_PAIR_SPLIT1 == 1) {
      x.par([&](int gl, Lane<W> &R) { phase_network<W, VARLOSS, ROLE_STAT>(gl, R, X, U, C, GlotOut{}); });
      x.mark(PH_S_GLOT);
      x.bar();
      x.mark(PH_P0WAIT);
      a_glot_up = X[X_AGLOT];
    } else if constexpr (kSplitA) {
      x.par_uniform([&](int gl, Lane<W> &R) { phase_network<W, VARLOSS, ROLE_STAT>(gl, R, X, U, C, GlotOut{}); },
                    [&](Lane<W> &R) {
                      (void)R;
                      a_glot_up = glottis_upper_area(glottis_inputs(X, rcur), ratio);
                    });
      x.mark(PH_S_GLOT);
    } else {
    x.par_uniform([&](int gl, Lane<W> &R) { phase_network<W, VARLOSS, ROLE_STAT>(gl, R, X, U, C, GlotOut{}); },
                  [&](Lane<W> &R) {
                    (void)R;
                    const double p4[4] = {X[X_P4 + 0], X[X_P4 + 1], X[X_P4 + 2], X[X_P4 + 3]};
                    GlotRes g;
                    if constexpr (Xc::kGlottisSplit && MODEL == AFS_GLOTTIS_TRIANGULAR)
                      g = glottis_eval_split(glottis_inputs(X, rcur), C, ratio, p4, x.half8(),
                                             [&](double v) { return x.xch8(v); });
                    else
                      g = glottis_eval<MODEL>(glottis_inputs(X, rcur), C, ratio, p4);
                    glottis_commit(X, g, rnext);
                    a_glot_up = g.go.a1;
                  });
    x.mark(PH_S_GLOT);
    }
    AFS_PM(";MARK targets");
#if !defined(AFS_PAIR_PROBE_NONOISE)
#if AFS_PAIR_RNG_DYN
    x.par([&](int gl, Lane<W> &R) {  // (the ring's head and pending count, which the DYN wave's rng_ahead moved)
      (void)gl;
      const int32_t *hp = (const int32_t *)(X + X_RNGHP);
      R.rhead = hp[0];
      R.rpend = hp[1];
    });
#endif
    x.par([&](int gl, Lane<W> &R) { phase_targets<W, NZ>(x, gl, R, X, C, a_glot_up); });
    x.sync();
    x.mark(PH_S_TGT);
    AFS_PM(";MARK noise");
    if (U.opt.generate_noise_sources) {
      phase_noise<W, NZ>(x, X, U, C);
    } else {
      x.par([&](int gl, Lane<W> &R) {
        (void)R;
        for (int d = gl; d < NDIP; d += W) X[X_SMP + d] = 0.0;
      });
    }
#if AFS_PAIR_RNG_DYN
    x.par([&](int gl, Lane<W> &R) {
      if (gl == 0) {
        int32_t *hp = (int32_t *)(X + X_RNGHP);
        hp[0] = R.rhead;
        hp[1] = R.rpend;
      }
    });
#endif
#endif
    x.mark(PH_NOISE);
  }
  x.bar();
  x.mark(PH_P1WAIT);
  if constexpr (ROLE == ROLE_STAT) {
    if (pair_prio(x) == 2) AFS_SETPRIO(0);
  }
  AFS_PM(";MARK rows");
  x.par([&](int gl, Lane<W> &R) { phase_rows<W, ROLE>(gl, R, X, X, U, C); });
  x.mark(PH_ROWS);
  x.bar();
  x.mark(PH_P2WAIT);
  AFS_PM(";MARK solver");
  if constexpr (ROLE == ROLE_STAT) {
    if (pair_prio(x) == 1 || pair_prio(x) == 2) AFS_SETPRIO(2);
  }
  if constexpr (ROLE == ROLE_STAT) {
#if !defined(AFS_PAIR_PROBE_NOSOLVE)
    // (64 lanes at one wave per SIMD: registers to spare for the full form)
    solve_arms<W, Xc, AFS_PAIR_LEAN != 0 && (W != 64 || AFS_PAIR64_WAVES >= 2)>(x, X, C);
#endif
    AFS_PM(";MARK rng");
#if !defined(AFS_PAIR_PROBE_NORNG) && !AFS_PAIR_RNG_DYN
    rng_ahead<W>(x, X);
#endif
  }
#if AFS_PAIR_RNG_DYN
  if constexpr (ROLE == ROLE_DYN) {  // the rand() blocks ahead on the DYN wave, beside the solver
    x.par([&](int gl, Lane<W> &R) {
      (void)gl;
      const int32_t *hp = (const int32_t *)(X + X_RNGHP);
      R.rhead = hp[0];
      R.rpend = hp[1];
    });
    rng_ahead<W>(x, X);
    x.par([&](int gl, Lane<W> &R) {
      if (gl == 0) {
        int32_t *hp = (int32_t *)(X + X_RNGHP);
        hp[0] = R.rhead;
        hp[1] = R.rpend;
      }
    });
    x.mark(PH_RNGP);
  }
#endif
  x.bar();
  x.mark(PH_P3WAIT);
  if constexpr (ROLE == ROLE_STAT) {
    if (pair_prio(x) == 1 || pair_prio(x) == 2) AFS_SETPRIO(0);
  }
  AFS_PM(";MARK update");
  if constexpr (ROLE == ROLE_DYN)
    x.par_uniform([&](int gl, Lane<W> &R) { phase_update<W, ROLE>(gl, R, X, X, U, C); },
                  [&](Lane<W> &R) { R.sample = phase_output_flow(X); });
  else
    x.par([&](int gl, Lane<W> &R) { phase_update<W, ROLE>(gl, R, X, X, U, C); });
  x.mark(PH_UPDATE);
  x.bar();
  x.mark(PH_P4WAIT);
}
template <int W, int MODEL, int NZ, int ROLE, class Xc>
AFS_HD inline void sample_step_pair(Xc &x, double *X, const Uni &U, const Consts &C, double ratio, int par) {
  if (U.opt.glottis_loss == AFS_ENTRANCE_LOSS_VARIABLE) sample_step_pair_v<W, MODEL, NZ, ROLE, true>(x, X, U, C, ratio, par);
  else sample_step_pair_v<W, MODEL, NZ, ROLE, false>(x, X, U, C, ratio, par);
}
#endif

}  // namespace tree
}  // namespace afs
