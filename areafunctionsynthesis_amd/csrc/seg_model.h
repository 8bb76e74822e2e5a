// seg_model.h -- tables of the segment-aligned synthesis kernel ("seg", afs_solver AFS_SOLVER_SEG;
// seg_core.h, tds_seg.hip), shared by host and device code.
//
// Sixteen lanes cooperate on one utterance, as in the tree kernel, but every lane owns the
// SAME currents in every phase of a sample -- network, matrix rows, elimination, state
// update -- so the 97-unknown system never goes through LDS (tools/seg_solver_study.py checks
// the elimination against a dense solve):
//
//  * dynamic part (the 50 currents whose rows change every sample: 23..69, 84, 93, 94): eleven
//    arm lanes with four positions each, in walk order (far end first), and a junction lane
//      arm A  [23 24 25 26] [27 28 29 30]+84 [31 32 33 34] [35 36 37 38]      (ascending)
//      arm B  [93 64 63 62]+94 [61 60 59 58] [57 56 55 54] [53 52 51 50] [49 48 47 46] [45 44 43 42]
//      arm C  [69 68 67 66]                                                       (descending)
//      junction lane [39 40 41 65]
//    (84 is folded on 28/29, 94 on 93/64: the fold slot has no interpolated geometry -- 84 is a
//    static section, 94 a radiation current); a lane walks its four positions in registers, the
//    boundaries are reduced lane to lane toward the junction by DPP, the junction lane solves
//    its four nodes, the solutions flow back;
//  * static part (the 47 currents whose two sections are static: trachea 0..22, nose 70..83
//    with the sinus leaves 89..92 and the nostril pair 95/96, fossa 85..88): their rows have
//    constant coefficients.  The three static subtrees hang from the dynamic currents 23, 69,
//    84 by one constant edge each, so their LDL^T is done once on the host: per sample a lane
//    needs only z = K^-1 y of its three chain positions and two leaf slots (a forward and a
//    backward linear recurrence with constant coefficients: a local sweep plus a four-step lane
//    scan each way); the attach node gets a constant pivot term and the right-hand side -e z_r,
//    and after the dynamic solve x = z - g x_d.
//
// Reference: the matrix is TdsModel::calcMatrix's (TdsModel.cpp:1785-2039); the reference
// factors it with an envelope Cholesky (:2231-2314); this is the exact LDL^T of the same
// matrix in another order (the tree kernel's arm solver is the same idea without the
// condensation).
#pragma once

#include <cstdint>

#include "afs_model.h"

namespace afs {
namespace seg {

constexpr int SW = 16;          // lanes per utterance (one DPP row)
constexpr int PD = 4;           // dynamic positions per lane
constexpr int NDS = PD + 1;     // dynamic slots: the four positions and the fold slot
constexpr int FOLD = PD;        // slot index of the fold
constexpr int PS = 3;           // static chain positions per lane
constexpr int NSS = PS + 2;     // static slots: chain positions and two leaf slots (on 0/1, 1/2)
constexpr int JUNCTION_LANE = 11;
constexpr int ARM_A_END = 3, ARM_B_END = 9, ARM_C_END = 10;  // lanes of the arms' last boundaries
constexpr int RED_STEPS = 5;    // sequential reduction steps of the longest arm (B: six lanes)
// static subtrees (trachea, nose, fossa): the lane and slot of the root, the attach current
constexpr int T_ROOT_LANE = 7, N_ROOT_LANE = 12, F_ROOT_LANE = 14;

// ---- per-utterance LDS block (doubles) ----------------------------------------------------
enum : int {
  SX_U = 0,                        // solution of the sample (currents), then zero, sink
  SX_U_ZERO = SX_U + NC, SX_U_SINK = SX_U_ZERO + 1,
  SX_UN = SX_U_SINK + 1,           // noise-smoothed flows (97), sink
  SX_UN_SINK = SX_UN + NC,
  SX_D = SX_UN_SINK + 1,           // D of every section, zero, sink
  SX_D_ZERO = SX_D + NS, SX_D_SINK = SX_D_ZERO + 1,
  SX_G = SX_D_SINK + 1,            // the section terms of the dynamic rows' sections: 22..69 and 84,
  NG = 49, G0 = 22,                //   8 doubles each (L, R1, E, D, area, 1/area, 1/r0, alpha), then a
                                   //   zero and a sink block
  SX_G_ZERO = SX_G + 8 * NG, SX_G_SINK = SX_G_ZERO + 8,
  SX_P4 = SX_G_SINK + 8,           // p[22..25] after the update (glottis inputs)
  SX_TVP = SX_P4 + 4,              // p[43], p[67] (transvelar filter inputs)
  SX_FRAME = SX_TVP + 2,           // teethL, teethR, velL, velR, gL[6], gR[6]
  SX_RELX = SX_FRAME + 16,         // glottis: cur0, cur1, prev0, prev1
  SX_GBF = SX_RELX + 4,
  SX_TONE = SX_GBF + 1,            // glottal tone filter x1..x4, y1..y4
  SX_OUTF = SX_TONE + 8,           // output Chebyshev x1..x8, y1..y8
  SX_PREVFLOW = SX_OUTF + 16,
  SX_NONFIN = SX_PREVFLOW + 1,
  SX_NDRAW = SX_NONFIN + 1,        // rand() calls so far (u64)
  SX_RNG = SX_NDRAW + 1,           // rand() value ring, prefix-sum ring, head, pending (65)
  SX_GP = SX_RNG + 65,             // interpolated glottis controls (6), 2 spare
  SX_TGLOT = SX_GP + 8,            // transglottal-pressure filter (variable entrance loss)
  SX_TVEL = SX_TGLOT + 8,          // transvelar coupling filters
  SX_ACT = SX_TVEL + 16,           // scratch / sinks of the noise phases (16)
  SX_FC = SX_ACT + 16,             // frame cache of the pharynx/mouth sections: aL, aR, lL, lR (40 x 4)
  SX_TOTAL = SX_FC + 4 * NPM,
  SX_STRIDE = SX_TOTAL + ((16 - SX_TOTAL % 32) + 32) % 32
};
static_assert(SX_STRIDE % 32 == 16, "utterance blocks offset by half a bank row");
static_assert(SX_G % 2 == 0, "16-byte aligned source blocks");
constexpr int GB = 8, G_L = 0, G_R1 = 1, G_E = 2, G_D = 3, G_AREA = 4, G_IAREA = 5, G_IR0 = 6, G_ALPHA = 7;
// the SX_G block of section s (-1: none)
AFS_HD constexpr int g_block(int s) {
  return (s >= G0 && s <= G0 + 47) ? SX_G + GB * (s - G0) : s == S_FOSSA0 ? SX_G + GB * 48 : -1;
}

// ---- dynamic slot records ------------------------------------------------------------------
// Where a slot's section area and length come from.
enum : uint8_t { K_NONE = 0, K_PM = 1, K_GLOT0 = 2, K_GLOT1 = 3, K_NOSE = 4, K_STATIC = 5 };
// Row and network flags of a dynamic slot.
enum : uint16_t {
  DF_CUR = 1,        // the slot holds a current (else a dummy: pivot 1, rhs 0)
  DF_SEC = 2,        // ... and the section it flows into (not a radiation current)
  DF_BIF = 4,        // the current's source section has two outputs (partner in this lane)
  DF_RAD_R = 8,      // radiation current R (93) / L (94) of section 64
  DF_RAD_L = 16,
  DF_JL = 32,        // Sondhi's inner length correction between pharynx/mouth sections
  DF_BERN = 64,      // Bernoulli pair (source, own section) can apply (TdsModel.cpp:850-877)
  DF_GLOT_R0 = 128,  // current 23: glottal entrance term on R0 of section 23
  DF_GLOT_R1 = 256,  // current 24: transition term on R1 of the source section 23
  DF_WALLS = 512,    // soft walls apply to the section (not the glottis)
  DF_RAD64 = 1024,   // the section is 64: radiation R and L of the mouth
  DF_TV67 = 2048,    // the section is 67: transvelar coupling source
  DF_FOSSA = 4096,   // the section is 84 (fossa entrance resistance option)
  DF_GLOTSEC = 8192, // the section is 23 or 24 (rmin 0.8, no walls)
  DF_LIPS = 16384    // the slot carries the lips dipole (fold of arm B's first lane)
};
struct alignas(16) DynSlot {
  uint16_t g_src;    // LDS byte offset of the source section's SX_G block (zero block: none)
  uint16_t g_own;    // where the slot publishes its section's SX_G block (sink: not 22..68)
  uint16_t d_own;    // SX_D slot of its section (sink: none)
  uint16_t out0, out1;  // SX_U slots of its section's output currents (zero: none)
  uint16_t u_pub;    // SX_U slot of its current (sink: none)
  uint16_t un_pub;   // SX_UN slot of its current (sink: none)
  uint16_t p_pub;    // SX_P4 / SX_TVP slot of its section's pressure (sink: none)
  uint16_t flags;
  uint8_t kind, m;   // area source; pharynx/mouth index (section - 25) for K_PM
  uint8_t dip;       // dipole 0..40 owned by the slot, 0xff: none
  uint8_t partner;   // slot of the bifurcation partner current (DF_BIF / radiation), 0xff
  uint8_t pad[2];
  double c0, c1;     // K_STATIC: area, length; K_NOSE: i*i / 16 (taper of nose section i)
};
static_assert(sizeof(DynSlot) == 48, "DynSlot: 48 bytes");

// Per lane: the walk and the condensation terms.
enum : uint8_t {
  WF_ASC = 1,        // positions in ascending current order (arm A): edge p-p+1 is the own
                     // section's, else the source section's
  WF_ANCHOR = 2,     // position 0 joins the previous lane's boundary
  WF_END = 4,        // last lane of an arm (its boundary joins a junction node)
  WF_JUNCTION = 8,   // the junction lane (no walk)
  WF_ARM = 16,       // an arm lane (walk, reduction)
  WF_FOLD_P0 = 32    // the fold's bifurcation partner is position q (else q + 1)
};
// the fold slot's section constants (a static section: 84; zeros for 94)
enum : int { FK_L, FK_R0, FK_R1, FK_E, FK_ALPHA, FK_K1, FK_K2, FK_K3, FK_N };
struct alignas(16) DynLane {
  uint8_t wf;        // WF_*
  uint8_t idx;       // position of the lane in its arm (0 = far end)
  uint8_t fold_q;    // the fold joins positions q, q+1 (0 or 1)
  uint8_t att0, attf;  // static subtree attached at position 0 / at the fold (0 none, 1 T, 2 N, 3 Fo)
  uint8_t pad[3];
  double delta0, e0;   // position 0's attach: constant pivot term, edge to the subtree root
  double deltaf, ef;   // the fold's
  double fk[FK_N];     // the fold's section (L, R0, R1, E, alpha, wall coefficients)
};
static_assert(sizeof(DynLane) == 112, "DynLane: 112 bytes");

// ---- static lanes -----------------------------------------------------------------------------
enum : uint16_t {
  SF_CUR = 1,        // the slot holds a current
  SF_SEC = 2,        // ... flowing into a section (not a nostril radiation current)
  SF_LUNG = 4,       // current 0: the lung pressure source (TdsModel.cpp:1989)
  SF_LIPS = 8,       // nostril radiation row: the lips dipole sample is its source term
  SF_ROOT = 16       // the subtree root (its z goes to the attach node)
};
// constants of one static slot (row coefficients and the update)
enum : int {
  SC_CU, SC_CUR, SC_CUD, SC_CUDR,   // H = -(cu u + cud uD) - (cur ur + cudr uDr) + S
  SC_E, SC_ALPHA, SC_K1, SC_K2, SC_K3,  // E; alpha; beta = k1 w + k2 wr + k3 wr2
  SC_INVD, SC_G, SC_CB,             // 1/D of the LDL^T; g of x = z - g x_d; back correction
  SC_N
};
struct alignas(16) StatSlot {
  uint16_t d_src;    // SX_D slot of the source section (zero: none)
  uint16_t d_own;    // SX_D slot of its section (sink: none)
  uint16_t out0, out1;
  uint16_t u_pub, un_pub, p_pub;
  uint16_t flags;
  uint16_t g_d;      // section 22 (the source of current 23): the D field of its SX_G block (sink: other)
  uint8_t partner;   // slot of the bifurcation partner (0xff: none)
  uint8_t pad[5];
  double c[SC_N];
};
static_assert(sizeof(StatSlot) % 16 == 0, "StatSlot: 16-byte multiple");
// per static lane: the chain multipliers and scan constants
enum : int {
  SL_FM0, SL_FM1, SL_FM2,           // forward multipliers into positions 0 (from the previous lane), 1, 2
  SL_FL00, SL_FL01, SL_FL11, SL_FL12,  // leaf multipliers: leaf 0 into positions 0, 1; leaf 1 into 1, 2
  SL_CF0, SL_CF1, SL_CF2,           // forward correction of positions 0..2 by the carry in
  SL_FQ0, SL_FQ1, SL_FQ2, SL_FQ3,   // forward scan products (levels 1, 2, 4, 8)
  SL_BM,                            // the next lane's forward multiplier into its position 0
  SL_BQ0, SL_BQ1, SL_BQ2, SL_BQ3,   // backward scan products
  SL_N
};
struct alignas(16) StatLane {
  uint8_t subtree;   // 0 none, 1 trachea, 2 nose, 3 fossa
  uint8_t root;      // slot of the subtree root in this lane (0xff: none)
  uint8_t pad[14];
  double k[SL_N];
  StatSlot s[NSS];
};

// network constants of the dynamic sections (walls of pharynx / mouth / nose sections)
enum : int { NK_INVK, NK_K1, NK_K2, NK_K3, NK_RRAD, NK_LRAD, NK_N = 8 };
struct SegConsts {
  DynSlot dyn[SW][NDS];
  DynLane dl[SW];
  StatLane st[SW];
  double nk[NK_N];
};

// The time loop's scalars (a copy of Tables::consts.h), staged in LDS next to the lane records.
struct SegHot {
  Hot h;
};

struct SegTables {
  SegConsts c;
  double g22[GB];     // the constant part of section 22's SX_G block (written at kernel start)
  SecRec uo[NS + 1];  // K5's view of the layout: x_uo0 / x_uo1 are SX_UN offsets (tree_plan.h)
  int32_t ok;         // the partition checks passed
};

// Host: the seg tables for the tube network of t (afs_seg_tables.cpp); ok = 0 when the
// partition does not use every current and edge exactly once.
void build_seg_tables(const Tables &t, SegTables *s);

}  // namespace seg
}  // namespace afs
