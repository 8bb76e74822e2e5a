// afs_model.h -- the branched-tube network shared by host and device code.
//
// Section/current numbering follows the reference exactly so that indices in tests
// and fixtures mean the same thing:
//   sections (Tube.h:53-82): 0-22 trachea, 23/24 glottis, 25-40 pharynx, 41-64 mouth,
//                            65-83 nose, 84-88 piriform fossa, 89-92 paranasal sinuses
//   currents (TdsModel.h:37, TdsModel.cpp:93-131): current c flows into section c
//                            (c < 93); 93/94 mouth radiation (R, L), 95/96 nostril radiation.
// Everything that does not change during synthesis -- static tube sections, their
// L/C/R/wall constants, filter coefficients, topology -- is evaluated once on the host
// (afs_tables.cpp) with the reference's own formulas and operand order, and handed to
// the kernels in one read-only `Tables` block.
#pragma once

#include <cstddef>
#include <cstdint>

#include "../../include/afs.h"

#if defined(__HIPCC__)
#define AFS_HD __host__ __device__
#else
#define AFS_HD
#endif

namespace afs {

constexpr int NS = 93;   // Tube::NUM_SECTIONS
constexpr int NC = 97;   // TdsModel::NUM_BRANCH_CURRENTS
constexpr int NPM = 40;  // pharynx + mouth sections
constexpr int S_LAST_TRACHEA = 22, S_GLOT_LO = 23, S_GLOT_UP = 24;
constexpr int S_PHARYNX0 = 25, S_LAST_PHARYNX = 40, S_MOUTH0 = 41, S_LAST_MOUTH = 64;
constexpr int S_NOSE0 = 65, S_LAST_NOSE = 83, S_FOSSA0 = 84, S_LAST_FOSSA = 88;
constexpr int S_SINUS0 = 89, S_LAST_SINUS = 92;
constexpr int NDIP = 41;  // dipole sources of sections 25..64, then the lips source
constexpr int DIP_LIPS = 40;
constexpr int ENV_COLS = 10;

enum Articulator : int { VOCAL_FOLDS = 0, TONGUE = 1, LOWER_INCISORS = 2, LOWER_LIP = 3, OTHER = 4 };

// Physical constants (Constants.h:8-16) and discretisation (TdsModel.cpp:15-22).
constexpr double RHO = 1.14e-3;
constexpr double CSND = 3.5e4;
constexpr double MU = 1.86e-4;
constexpr double TH = 0.515;
constexpr double TH1 = 1.0 - 0.515;
constexpr double AMIN = 0.1e-2;
constexpr double PI = 3.14159265358979323846;

// Glottis static parameters (TriangularGlottis.cpp:38-56).
constexpr double G_REST_LEN = 1.3, G_REST_THICK0 = 0.24, G_REST_THICK1 = 0.06;
constexpr double G_MASS0 = 0.12, G_MASS1 = 0.03, G_DAMP0 = 0.1, G_DAMP1 = 0.6;
constexpr double G_K0 = 80000.0, G_K1 = 8000.0, G_KC0 = 240000.0, G_KC1 = 24000.0;
constexpr double G_KCOUPLE = 25000.0, G_INLET = 0.05, G_OUTLET = 0.01;
constexpr double G_NAT_F0 = 129.0, G_F0_DIV_Q = 125.51;
// TwoMassModel static parameters (TwoMassModel.cpp:36-58).
constexpr double TM_REST_LEN = 1.3, TM_REST_THICK0 = 0.25, TM_REST_THICK1 = 0.05;
constexpr double TM_MASS0 = 0.125, TM_MASS1 = 0.025, TM_DAMP0 = 0.1, TM_DAMP1 = 0.6;
constexpr double TM_K0 = 80000.0, TM_K1 = 8000.0, TM_ETA0 = 100.0, TM_ETA1 = 100.0;
constexpr double TM_KC0 = 240000.0, TM_KC1 = 24000.0, TM_CETA0 = 500.0, TM_CETA1 = 500.0;
constexpr double TM_KCOUPLE = 25000.0, TM_CRIT_WIDTH = 0.0, TM_NAT_F0 = 158.0, TM_F0_DIV_Q = 100.0;
constexpr double TM_CHINK_LEN = 0.2;
constexpr double GLOTTIS_DEFAULT_ASPIRATION_DB = -40.0;  // Glottis.cpp:5

// A section is "static" when nothing about its geometry changes during synthesis:
// trachea, nose beyond the velum taper (nose[4..18]), fossa, sinuses.
AFS_HD constexpr bool is_static_section(int s) {
  return s <= S_LAST_TRACHEA || (s >= S_NOSE0 + 4);
}

// Edges of the current graph (afs_tables.cpp edge_numbering): for section s with in-current
// a and out-currents b (c), edge[s][0] = (a,b), edge[s][1] = (a,c), edge[s][2] = (b,c);
// TREE_NE of them, each with its own LDS slot.
constexpr int TREE_CHAINS = 16;  // lanes of the per-sample solver
constexpr int TREE_NE = 104;
// Arm solver (tree_core.h solve_arms; afs_tables.cpp arm_records).  The current graph is a
// junction triangle {40, 41, 65} with three arms (A: 0..39 with the fossa 84..88 on {28, 29};
// B: 42..64 with the radiation pair 93/94; C: 66..83 with the pair 95/96 and the sinus leaves
// 89..92).  Each of the 16 lanes owns a segment of an arm at positions 0..ARM_P-1, right
// aligned (its last node, the lane's boundary, at ARM_P-1; dummy positions in front), folds
// the leaves of its segment (fold slot f joins a leaf to positions ARM_FOLD_POS[f] and +1),
// eliminates the segment's other nodes in registers, and the boundaries are reduced lane to
// lane by DPP.  Lane roles are fixed by the partition: the fossa lane folds 84 into the
// boundaries 28 / 29 of ARM_L28 / ARM_L28 + 1, the junction lane solves the triangle.
constexpr int ARM_P = 8, ARM_FOLDS = 4, ARM_MAXLEN = 7;  // ARM_MAXLEN: lanes of the longest arm
// a segment's first real position is at most ARM_START_MAX, or ARM_P - 1 (a one-node segment,
// its boundary) or ARM_P (none): the walk sets its anchor edge only at positions up to it
constexpr int ARM_START_MAX = 3;
constexpr int ARM_FOSSA = 14, ARM_JUNCTION = 15, ARM_L28 = 3;
constexpr int ARM_END_A = 6, ARM_END_B = 10, ARM_END_C = 13;  // lanes of the arms' last boundaries
AFS_HD constexpr int arm_fold_pos(int f) { return f == 0 ? 2 : f == 1 ? 3 : f == 2 ? 5 : 6; }
enum : uint8_t { ARM_IN = 1, ARM_END = 2 };
// LDS byte offsets (utterance block) of one lane's part; dummy positions and unused fold
// slots point at the ONE pivot slot (1.0, rhs 0.0), the zero edge and the solution sink, so
// that every lane runs the same code and a dummy step changes nothing.
struct alignas(16) ArmRec {
  uint16_t d[ARM_P];          // pivot (X_DIAG) of position p; its rhs at RHS_DELTA
  uint16_t u[ARM_P];          // X_U slot of position p: its fill edge to the anchor, then x
  uint16_t e[ARM_P - 1];      // edge p - p+1 (X_OFF)
  uint16_t ea;                // edge anchor (previous lane's boundary) - first real node
  uint16_t ld[ARM_FOLDS], le0[ARM_FOLDS], le1[ARM_FOLDS], lu[ARM_FOLDS];  // fold leaves
  uint16_t fx0, fx1;          // fossa lane: edges 84-28, 84-29 (else the zero edge)
  uint16_t ej;                // last lane of an arm: edge boundary - junction node
  uint8_t start;              // first real position (ARM_P: none)
  uint8_t idx, flags, pad0;   // position in the arm (0 = far end), ARM_IN / ARM_END
  uint16_t pad[11];
  // (112-byte stride, 7 x 16: the 16 lanes of an utterance read records 0-15, which then start on
  // 16 distinct 16-byte bank slots; at 96 bytes lanes k and k + 8 shared them, 2-way conflicts)
};
static_assert(sizeof(ArmRec) == 112, "ArmRec: 112 bytes");
// the junction triangle: pivots of 40, 41, 65, edges 40-41, 40-65, 41-65, X_U of 40, 41, 65
struct alignas(8) ArmJunction {
  uint16_t d[3], e[3], u[3], pad;
};
// Currents whose d/dt another lane reads (branch partners and radiation; tree_core.h X_UR).
constexpr int NUR = 16;
// Currents whose noise-filtered value another lane reads (outputs of the constriction
// candidates 24..64 and the radiation currents; tree_core.h X_UN).
constexpr int NUN = 48;

// The tables the cooperative kernel reads inside its time loop, packed so that one copy
// per wave fits in LDS next to the four utterance blocks (tds_tree.hip).
constexpr int NSTATIC = 47;  // static sections 0..22, 69..92 -> index s < 23 ? s : s - 46
enum : int { ST_E, ST_ALPHA, ST_WC1, ST_WC2, ST_LW, ST_L, ST_R, ST_N };
// Per section s (= per current i = s flowing into it): source section of the current, the
// other output current of that source (its bifurcation partner, -1: none) and that
// partner's X_UR slot, the section's output currents and its edges.  8 bytes: one load.
struct alignas(8) Topo {
  int8_t src, br, urbr, out0, out1, e0, e1, e2;
};
// Per section s (index NS: an absent slot), the LDS doubles of the utterance block that the
// matrix row of its in-current and its state update touch besides its own section, as
// indices into the block (tree_core.h layout).  Absent neighbours point at the zero slot
// (reads) or the sink slot (writes), so the phases load one record per slot and branch only
// on the row kind.
//   row:    x_la/x_ra/x_ea = L, R1, E of the source section when it is dynamic (X_L, X_R1,
//           X_E), c_la/c_ra/c_ea the same constants when it is static (else 0.0); x_da = its
//           D; x_ub/x_urb = flow and d/dt of the bifurcation partner; x_sx = the source term
//           (dipole sample, lung pressure); x_e0..x_e2 = the section's edges (X_OFF).
//   update: x_o0/x_o1 = flows of the output currents; x_ur/x_un/x_p4 = where d/dt and the
//           noise-smoothed value of the in-current and the pressure are published.
enum : uint16_t { SR_BIF = 1, SR_JUNCTION = 2, SR_RADIATION = 4 };
// (The x_* fields are LDS byte offsets into the utterance block: the kernel adds them to the
// block's address with one instruction, sub-dword operand select included.)
// Fields grouped by the phase that reads them, each group at an offset aligned to its load width:
// the compiler merges adjacent 16-bit fields into one wide LDS read, and a read that is not
// aligned to its width stalls the LDS (SQ_LDS_UNALIGNED_STALL; the previous order had the row
// phase's offsets in a 12-byte read at byte 30 of the record).
struct alignas(16) SecRec {
  uint16_t x_la, x_da, x_ub, x_urb, x_sx, x_e0, x_e1, x_e2;  // row phase (bytes 0-15)
  double c_la, c_ra, c_ea;                                    // row phase (16-39)
  uint16_t flags;
  // constriction phase: the noise-smoothed flows of the section's outputs (X_UN, or zero)
  uint16_t x_uo0, x_uo1;
  uint16_t x_ra;                                              // (unused by the kernel)
  uint16_t x_o0, x_o1, x_ur, x_un, x_p4;                      // update phase (48-57)
  uint16_t x_ea, pad0[2];                                     // (x_ea unused by the kernel)
  // radiation sections (SR_RADIATION): flow, d/dt and noise-smoothed flow of the two
  // radiation currents (X_U + rc, X_U + lc, X_UR.., X_UR.., X_UN.., X_UN..) (64-75)
  uint16_t x_rad[6];
  uint16_t pad1[2];
  // (80-byte stride: the 16 sections a 16-lane ds_read_b128 group reads start on 16 distinct
  // 16-byte bank slots; at 64 bytes, sections s and s+4 share banks: 4-way conflicts)
};
static_assert(offsetof(SecRec, c_la) == 16 && offsetof(SecRec, x_o0) == 48 && offsetof(SecRec, x_rad) == 64,
              "SecRec: the phases' field groups at aligned offsets");
static_assert(sizeof(SecRec) == 80, "SecRec: 80-byte stride");
// Scalars of the time loop (copies of Tables fields; see build_tables).
struct Hot {
  double fs, dt, dtTH1, noise_amp_F, noise_lp_c, noise_x_2000, sqrt12, nose4_area, fossa_R0;
  double rrad_num, lrad_num, tone_a[5], tone_b[5], out_a[9], out_b[9];
  double len_nose0, Bw_ph0, Mw_ph0, Kw_ph0, area_last_trachea, area_last_nose;
  double rrad_nose, lrad_nose;  // radiation R and L of the nostrils (static section 83)
  double inv_dtTH, inv_dt2TH2;  // 1 / (dt theta), 1 / (dt theta)^2
  double Tt;                    // glottis time step 1 / fs
  double inv_dt;                // 1 / dt
  double g_smk0, g_smk1;        // sqrt(mass * stiffness) of the two glottis masses (q-free)
  double tglot_a[5], tglot_b[5];  // transglottal-pressure Chebyshev, 50 Hz (TdsModel.cpp:474)
  double tvel2_a[5];              // transvelar coupling H2 numerator (H1 = tone_a; b = tone_b)
  // the walls of the dynamic sections with the wall surface cancelled: alpha = surf * wall_invK,
  // beta = wall_k1 w + wall_k2 w' + wall_k3 w'' (TdsModel.cpp:805-832); the mouth's radiation
  // elements Rrad = rrad_c / A, Lrad = lrad_c r0 / A (:1874, :1889)
  double wall_invK, wall_k1, wall_k2, wall_k3, rrad_c, lrad_c;
  // per glottis mass i: mass, stiffness, contact stiffness, damping ratio, sqrt(mass stiffness),
  // inlet / outlet factor, rest thickness (the constants of TriangularGlottis::incTime for the
  // mass a lane evaluates when the masses are split over an utterance's lanes, tree_core.h);
  // 256 B with the padding, so the LDS blocks after the tables keep their bank alignment
  double gmass[2][8];
  double gmass_pad[16];
};
// Values that steer branches in the time loop: kernel arguments on the device, so the
// compiler keeps them in scalar registers and branches on them uniformly.
struct Uni {
  afs_options opt;
};
struct Consts {
  Hot h;
  ArmRec arm[TREE_CHAINS];
  ArmJunction armj;
  int8_t ur_slot[NC];  // X_UR slot of a current, -1: none
  int8_t un_slot[NC];  // X_UN slot of a current, -1: none
  Topo topo[NS];
  double stat[NSTATIC][ST_N];
  SecRec sec[NS + 1];
};

struct Tables {
  // time step and derived scalars
  double fs, dt, dtTH, dtTH1, th1_th, inv_dtTH;
  double noise_amp_F;      // 1 - exp(-2 pi 40 dt)           (TdsModel.cpp:1637-1638)
  double noise_lp_c;       // exp(-2 pi 500 dt)               (TdsModel.cpp:2061)
  double noise_x_2000;     // exp(-2 pi (2000 dt)): one-pole coefficient at the clamped cutoff
  double sqrt12;           // sqrt(12.0)
  double nose4_area;       // Tube noseSection[4].area, target of the velum taper (Tube.cpp:407)
  double fossa_R0;         // decoupled fossa entrance resistance (TdsModel.cpp:888)
  double rrad_num, lrad_num; // 128 rho c, 8 rho                     (TdsModel.cpp:1874, 1889)
  double tone_a[5], tone_b[5];  // glottalToneFilter (TdsModel.cpp:494-510)
  double out_a[9], out_b[9];    // Chebyshev(7000/fs, 8 poles)     (Synthesizer.cpp:52)
  double tglot_a[5], tglot_b[5];  // Chebyshev(50/fs, 4 poles)      (TdsModel.cpp:474)
  double tvel2_a[5];            // transvelar coupling filter 2     (TdsModel.cpp:511-524)

  // per-section geometry and walls (static sections: final values; dynamic: walls only)
  double area[NS], len[NS], vol[NS], Mw[NS], Bw[NS], Kw[NS];
  // static-section network constants, evaluated as prepareTimeStep would (TdsModel.cpp:732-834)
  double L[NS], C[NS], R[NS], alpha[NS], wc1[NS], wc2[NS], Lw[NS], E[NS];

  // topology (TdsModel::initModel, TdsModel.cpp:93-292)
  int16_t src[NC], tgt[NC], cin[NS], cout0[NS], cout1[NS];
  // symmetric-envelope Cholesky structure: row i spans columns env_start[i] .. i-1
  int16_t env_start[NC], env_n[NC], env_off[NC];
  int16_t col_n[NC], col[NC][ENV_COLS];
  int32_t env_total;
  // SOR rows: filledRowIndex (TdsModel.cpp:340-357), ascending columns, at most 16
  int16_t row_n[NC], row[NC][16];

  // tree solver: edge numbering; n_rounds = the arm solver's sequential reduction steps
  // (ARM_MAXLEN - 1), -1 when the tables fail their checks
  int16_t edge[NS][3];
  int32_t n_edges, n_rounds;
  Consts consts;
  Uni uni;

  afs_options opt;
};

// TdsModel's default options (TdsModel.cpp:35-44).
inline afs_options default_options() {
  afs_options o{};
  o.turbulence_losses = 1;
  o.soft_walls = 1;
  o.generate_noise_sources = 1;
  o.radiation_from_skin = 1;
  o.piriform_fossa = 0;
  o.inner_length_corrections = 1;
  o.transvelar_coupling = 0;
  o.glottis_loss = AFS_ENTRANCE_LOSS_STANDARD;
  o.glottis_model = AFS_GLOTTIS_TRIANGULAR;
  o.flow_separation_area_ratio = 1.0;
  return o;
}

// Host: build the tables for a sampling rate and option set (afs_tables.cpp).
void build_tables(Tables *t, double fs_hz, const afs_options &opt);
// Host: IirFilter::createChebyshev restatement used for the output filter.
int chebyshev(double ratio, bool highpass, int poles, double *a, double *b);

}  // namespace afs
