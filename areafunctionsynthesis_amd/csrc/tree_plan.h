// tree_plan.h -- the noise-source plan of one audio sample (kernel K5, tds_plan.hip).
//
// Everything calcNoiseSources (src/Backend/TdsModel.cpp:1188-1604) decides from the tube
// GEOMETRY alone -- which constrictions exist (glottis, up to two tongue constrictions, the
// lower lip), their extent, laterality, obstacle position, the two dipole sources each one
// drives, the source weights and the area terms of the narrowest section -- depends only on
// the interpolated frame of that sample (Tube::interpolate, Tube.cpp:438-505, and
// Tube::calcPositions, :579-654), not on the acoustic state.  K5 evaluates it for every
// utterance-sample ahead of the time loop, one thread per sample, with the reference's own
// sequential scans; the cooperative synthesis kernel then reads 128 bytes per sample and
// only combines them with the state-dependent flows (TdsModel.cpp:1507-1602).  This takes
// the constriction scans -- ballots and lane reductions over the 40 pharynx/mouth sections,
// a quarter of the per-sample latency chain -- out of the recurrence.
//
// The same function runs on the host (tests/emu), so the CPU emulator checks the split
// against the oracle.
#pragma once

#include <cstdint>

#include "afs_model.h"

#if !defined(__HIPCC__)
#include <cmath>
#endif

namespace afs {
namespace tree {

// One record = 16 u64 words; word w is held by lane w of the utterance in the synthesis
// kernel and broadcast to the other lanes (DPP row_newbcast) where it is used.
enum : int {
  PW_HDR = 0,     // bytes 0..4: flags, up of glottis / tongue 1 / tongue 2 / lip (0..39)
  PW_UO = 1,      // u16 x 4: X_UN byte offsets of the outputs of the narrowest section, tongue 1, 2
  PW_UOL = 2,     // u16 x 2: the same for the lip constriction
  PW_FDN = 3,     // 4 words: downstream factor of glottis, tongue 1, tongue 2, lip
  PW_T1 = 7,      // 3 words: 1/A, sqrt(A), 1/d of the narrowest section (A >= 0.1, d = sqrt(4A/pi))
  PW_T2 = 10,     // 3 words: the same for tongue 2
  PW_L = 13,      // 2 words: 1/A, sqrt(A) of the lip constriction
  PW_GAIN_G = 15, // glottis dipole gain 0.5e-7 * 10^(aspiration dB / 20) (TdsModel.cpp:1546)
  PLAN_WORDS = 16
};
enum : uint32_t {
  PF_G = 1, PF_T1 = 2, PF_T2 = 4, PF_L = 8,  // constriction present and its obstacle section found
  PF_T1_LAT = 16, PF_T2_LAT = 32,           // laterality > 0.1: full amplitude 0 (:1567-1571)
  PF_T1_TEETH = 64, PF_T2_TEETH = 128       // obstacle at the teeth: gain 10e-7, else 5e-7 (:1549-1562)
};

AFS_HD inline uint64_t plan_bits(double v) {
#if defined(__HIPCC__)
  return __builtin_bit_cast(uint64_t, v);
#else
  uint64_t b;
  __builtin_memcpy(&b, &v, 8);
  return b;
#endif
}
AFS_HD inline double plan_double(uint64_t b) {
#if defined(__HIPCC__)
  return __builtin_bit_cast(double, b);
#else
  double v;
  __builtin_memcpy(&v, &b, 8);
  return v;
#endif
}

AFS_HD inline double plan_clampA(double a) { return a < AMIN ? AMIN : a; }
// The scans over the 40 sections unrolled twice: fully unrolled they hold 134 VGPRs with the
// pre-clamped areas (K5: 57 at unroll 2, 30.5 vs 35.8 ms per step of 8192 utterances x 1 s,
// DESIGN.md 4).
#define PLAN_LOOP _Pragma("unroll 2")

// The interpolated pharynx/mouth geometry of one sample, evaluated on demand (no per-thread
// arrays: K5 keeps its registers for occupancy).  Every value is computed with the operations
// of tree_core.h phase_interpolate and Tube::calcPositions, with contraction into fmas off in
// both (the pragmas below and in phase_interpolate), so K5 and the synthesis kernel see the same
// bits whatever the compiler's -ffp-contract default, and re-evaluation gives the same value.
template <bool PRE>  // PRE: the frames' areas are clamped already (K5's LDS copy)
struct PlanGeomT {
  using V = double;
  const afs_frame *fl, *fr;
  double r1, ratio;
  AFS_HD double area(int m) const {
#pragma clang fp contract(off)
    if constexpr (PRE) return plan_clampA(r1 * fl->area_cm2[m] + ratio * fr->area_cm2[m]);
    return plan_clampA(r1 * plan_clampA(fl->area_cm2[m]) + ratio * plan_clampA(fr->area_cm2[m]));
  }
  AFS_HD double len(int m) const {
#pragma clang fp contract(off)
    return r1 * fl->length_cm[m] + ratio * fr->length_cm[m];
  }
  AFS_HD double lat(int m) const {
#pragma clang fp contract(off)
    return r1 * fl->laterality[m] + ratio * fr->laterality[m];
  }
  AFS_HD double teeth() const {
#pragma clang fp contract(off)
    return r1 * fl->teeth_position_cm + ratio * fr->teeth_position_cm;
  }
  AFS_HD int art(int m) const { return fl->articulator[m]; }  // the left tube's (Tube.cpp:452)
  AFS_HD double pos0() const { return 0.0; }                  // the running position sums' start
  // the decisions' comparisons
  AFS_HD static bool lt(double a, double b) { return a < b; }
  AFS_HD static bool le(double a, double b) { return a <= b; }
};

// ---------------------------------------------------------------------------
// The same geometry over a range of samples of one hop (ratios i / hop, i = i0 .. i1-1), as
// intervals that contain every value a sample of the range computes (K5's hop mode decides a
// whole hop with one evaluation when every comparison of plan_decide is decided for all of
// them).  Each interpolated value (1 - r) a + r b lies, for every sample, within
// 2^-50 (|a| + |b|) of the interval spanned by the two end samples' own values (the exact
// interpolation is monotone in r, the rounding of r, 1 - r, the products and the sum is below
// that); sums and differences widen by 2^-51 of their magnitude.  Identical quantities -- the same
// section's interpolated area or laterality (same inputs), the running position sums of the
// position and obstacle passes -- carry an identity, so that they compare equal exactly (a tie
// in the scans, the lip obstacle at the end of its own section).
// ---------------------------------------------------------------------------
struct PlanIv {
  double lo, hi;
  int kind;     // identity: IV_NONE, or what the value is (the same kind and inputs: equal everywhere)
  double a, b;  // IV_AREA / IV_LAT / IV_TEETH: the interpolation's inputs; IV_POS / IV_LEN: the index
  PlanIv() = default;
  AFS_HD explicit PlanIv(double c) : lo(c), hi(c), kind(0), a(0.0), b(0.0) {}
  AFS_HD PlanIv(double lo_, double hi_, int kind_, double a_, double b_) : lo(lo_), hi(hi_), kind(kind_), a(a_), b(b_) {}
};
enum : int { IV_NONE = 0, IV_AREA = 1, IV_POS = 2, IV_LEN = 3, IV_LAT = 4, IV_TEETH = 5 };
AFS_HD inline PlanIv plan_iv(double c) { return PlanIv(c); }
AFS_HD inline bool plan_iv_same(const PlanIv &x, const PlanIv &y) {
  return x.kind != IV_NONE && x.kind == y.kind && x.a == y.a && x.b == y.b;
}
AFS_HD inline PlanIv plan_iv_widen(double lo, double hi) {
  const double e = 4.440892098500626e-16;  // 2^-51
  return PlanIv{lo - fabs(lo) * e, hi + fabs(hi) * e, IV_NONE, 0.0, 0.0};
}
AFS_HD inline PlanIv operator+(const PlanIv &x, const PlanIv &y) {
  PlanIv r = plan_iv_widen(x.lo + y.lo, x.hi + y.hi);
  if (x.kind == IV_POS && y.kind == IV_LEN && x.a == y.a) {  // pos[m] + len[m] = pos[m + 1]
    r.kind = IV_POS;
    r.a = x.a + 1.0;
  }
  return r;
}
AFS_HD inline PlanIv &operator+=(PlanIv &x, const PlanIv &y) { return x = x + y; }
AFS_HD inline PlanIv operator+(const PlanIv &x, double c) { return plan_iv_widen(x.lo + c, x.hi + c); }
AFS_HD inline PlanIv operator*(double c, const PlanIv &x) {  // (c >= 0)
  return plan_iv_widen(c * x.lo, c * x.hi);
}
AFS_HD inline PlanIv operator-(const PlanIv &x, const PlanIv &y) {
  if (plan_iv_same(x, y)) return plan_iv(0.0);
  return plan_iv_widen(x.lo - y.hi, x.hi - y.lo);
}
AFS_HD inline double plan_abs(double x) { return fabs(x); }
AFS_HD inline PlanIv plan_abs(const PlanIv &x) {
  if (x.lo >= 0.0) return x;
  if (x.hi <= 0.0) return PlanIv{-x.hi, -x.lo, IV_NONE, 0.0, 0.0};
  return PlanIv{0.0, -x.lo > x.hi ? -x.lo : x.hi, IV_NONE, 0.0, 0.0};
}

template <bool PRE>
struct PlanGeomIv {
  using V = PlanIv;
  const afs_frame *fl, *fr;
  double r1lo, rlo, r1hi, rhi;  // the end samples' 1 - r and r
  mutable int undecided;        // a comparison that is not the same for every sample of the range
  AFS_HD PlanIv lerp(double a, double b, int kind, bool clamp) const {
#pragma clang fp contract(off)
    const double u0 = r1lo * a + rlo * b, u1 = r1hi * a + rhi * b;
    const double w = (fabs(a) + fabs(b)) * 8.881784197001252e-16;  // 2^-50
    double lo = (u0 < u1 ? u0 : u1) - w, hi = (u0 < u1 ? u1 : u0) + w;
    if (clamp) {
      lo = plan_clampA(lo);
      hi = plan_clampA(hi);
    }
    return PlanIv{lo, hi, kind, a, b};
  }
  AFS_HD PlanIv area(int m) const {
    const double a = PRE ? fl->area_cm2[m] : plan_clampA(fl->area_cm2[m]);
    const double b = PRE ? fr->area_cm2[m] : plan_clampA(fr->area_cm2[m]);
    return lerp(a, b, IV_AREA, true);
  }
  AFS_HD PlanIv len(int m) const {
    PlanIv v = lerp(fl->length_cm[m], fr->length_cm[m], IV_LEN, false);
    v.a = (double)m;
    v.b = 0.0;
    return v;
  }
  AFS_HD PlanIv lat(int m) const { return lerp(fl->laterality[m], fr->laterality[m], IV_LAT, false); }
  AFS_HD PlanIv teeth() const { return lerp(fl->teeth_position_cm, fr->teeth_position_cm, IV_TEETH, false); }
  AFS_HD int art(int m) const { return fl->articulator[m]; }
  AFS_HD PlanIv pos0() const { return PlanIv{0.0, 0.0, IV_POS, 0.0, 0.0}; }
  AFS_HD bool lt(const PlanIv &x, const PlanIv &y) const {
    if (plan_iv_same(x, y)) return false;
    if (x.hi < y.lo) return true;
    if (x.lo >= y.hi) return false;
    undecided = 1;
    return false;
  }
  AFS_HD bool le(const PlanIv &x, const PlanIv &y) const {
    if (plan_iv_same(x, y)) return true;
    if (x.hi <= y.lo) return true;
    if (x.lo > y.hi) return false;
    undecided = 1;
    return false;
  }
  AFS_HD bool lt(const PlanIv &x, double c) const { return lt(x, plan_iv(c)); }
};

// first section with the articulator and the smallest area (strict "<", from 1e6), -1: none
template <class G>
AFS_HD inline int plan_argmin(const G &g, int a, typename G::V &amin, int skip_lo = 1, int skip_hi = 0) {
  using V = typename G::V;
  int n = -1;
  amin = V(1000000.0);
  PLAN_LOOP
  for (int m = 0; m < NPM; ++m) {
    const V A = g.area(m);
    if (g.art(m) == a && (m < skip_lo || m > skip_hi) && g.lt(A, amin)) { amin = A; n = m; }
  }
  return n;
}
// the reference's constriction extent (TdsModel.cpp:1247-1262): from the narrowest section
// outwards while the area stays below amin + 0.2 with the same articulator, then one back
template <class G>
AFS_HD inline void plan_grow(const G &g, int narrow, const typename G::V &amin, int a, int &first, int &last) {
#pragma clang fp contract(off)
  using V = typename G::V;
  const V maxA = amin + 0.2;
  first = narrow;
  last = narrow;
  while (g.lt(g.area(first), maxA) && g.art(first) == a && first > 0) --first;
  while (g.lt(g.area(last), maxA) && g.art(last) == a && last < NPM - 1) ++last;
  ++first;
  --last;
}
template <class G>
AFS_HD inline typename G::V plan_max_lat(const G &g, int first, int last) {
  using V = typename G::V;
  V l = V(0.0);
  for (int m = first; m <= last; ++m)
    if (g.lt(l, g.lat(m))) l = g.lat(m);
  return l;
}

// The discrete decisions of one sample's plan: which sections are the narrowest ones, where the
// constrictions end, which obstacle formula applies and in which section each obstacle lies.
// Everything else in the record is a continuous function of the interpolated geometry.
struct PlanKey {
  int n1, n2, nl;   // narrowest tongue section, second tongue constriction's, lower lip's (-1: none)
  int l1, l2, ll;   // last sections of the three extents (-1: none)
  int mo[4];        // obstacle section of glottis, tongue 1, tongue 2, lip (-1: none)
  bool has_t1, has_t2, lip_c, has_l;
  bool tb1, tb2;    // the tongue obstacle is the teeth (:1283-1299)
  uint32_t flags;   // PF_*
};
// The dipole sources a sample's decisions target -- bit d for dipole d (0..40: the up- and
// downstream source of every constriction present, TdsModel.cpp:1590-1604; a lateral tongue
// constriction targets its sources with amplitude 0) -- and, bits NOISE_CON0 + c, the
// constrictions present (PF_G, PF_T1, PF_T2, PF_L).
constexpr int NOISE_CON0 = 48;
AFS_HD inline uint64_t plan_key_noise(const PlanKey &k) {
  uint64_t m = 0;
  for (int c = 0; c < 4; ++c)
    if (k.flags & (1u << c)) {
      const int up = k.mo[c], dn = up < NPM - 1 ? up + 1 : DIP_LIPS;
      m |= (1ull << up) | (1ull << dn) | (1ull << (NOISE_CON0 + c));
    }
  return m;
}
// The noise-phase variant classes of the 16-lane synthesis kernel (tree_core.h NoiseV): the
// plan_key_noise bits the glottis-only variant serves (the glottis constriction, dipoles 0-15: its
// lanes' first slot) and the glottis + first tongue constriction variant (dipoles 0-31).  Class 2,
// 1 or 0 (the full phases) of a mask; the slot order groups utterances by the class of their first
// frame (afs_capi.cpp shape_order).
constexpr uint64_t NOISE_SERVES16_GLOTTIS = (1ull << NOISE_CON0) | 0xFFFFull;
constexpr uint64_t NOISE_SERVES16_TONGUE1 = (3ull << NOISE_CON0) | 0xFFFFFFFFull;
constexpr uint64_t NOISE_SERVES16_T1ALL = (3ull << NOISE_CON0) | ((1ull << NOISE_CON0) - 1);
AFS_HD inline int plan_noise_class16(uint64_t m, int set) {  // set: the variants compiled (AFS_NZ_SET)
  if ((set & 2) && (m & ~NOISE_SERVES16_GLOTTIS) == 0) return 3;
  if ((set & 1) && (m & ~NOISE_SERVES16_TONGUE1) == 0) return 2;
  return ((set & 4) && (m & ~NOISE_SERVES16_T1ALL) == 0) ? 1 : 0;
}
// Two 64-bit words that are equal iff the keys are.
AFS_HD inline void plan_key_pack(const PlanKey &k, uint64_t *q) {
  auto b6 = [](int v) { return (uint64_t)(uint32_t)(v + 1) & 63u; };  // -1 .. 62
  q[0] = b6(k.n1) | b6(k.n2) << 6 | b6(k.nl) << 12 | b6(k.l1) << 18 | b6(k.l2) << 24 | b6(k.ll) << 30 |
         b6(k.mo[0]) << 36 | b6(k.mo[1]) << 42 | b6(k.mo[2]) << 48 | b6(k.mo[3]) << 54;
  q[1] = (uint64_t)k.flags | (uint64_t)k.has_t1 << 8 | (uint64_t)k.has_t2 << 9 | (uint64_t)k.lip_c << 10 |
         (uint64_t)k.has_l << 11 | (uint64_t)k.tb1 << 12 | (uint64_t)k.tb2 << 13;
}

// The discrete decisions at one sample (g: its interpolated geometry; PlanGeomT) or, with the
// interval geometry PlanGeomIv, for every sample of a range at once (valid unless g.undecided),
// and the obstacle positions / the positions of the obstacle sections that go into the
// downstream factors.
// The reference's scans (argmin, extent, position, obstacle) are merged into four passes over
// the 40 sections: the narrowest tongue and lip sections together, the second tongue
// constriction, one running position sum for every position the obstacles need, and one
// obstacle search for all four constrictions.  Every value is the one the separate scans give
// (the same comparisons and the same sequential sums).
template <class G>
AFS_HD inline void plan_decide(const G &g, PlanKey &key, typename G::V *obst, typename G::V *po) {
#pragma clang fp contract(off)
  using V = typename G::V;
  const V teeth = g.teeth();
  // narrowest tongue section (:1228-1240) and narrowest lower-lip section (:1399-1410): the
  // first strict minimum from 1e6
  int n1 = -1, nl = -1;
  V amin1 = V(1000000.0), aminl = V(1000000.0);
  PLAN_LOOP
  for (int m = 0; m < NPM; ++m) {
    const V A = g.area(m);
    const int a = g.art(m);
    if (a == TONGUE && g.lt(A, amin1)) { amin1 = A; n1 = m; }
    if (a == LOWER_LIP && g.lt(A, aminl)) { aminl = A; nl = m; }
  }
  // tongue constriction 1 (:1228-1302)
  const bool has_t1 = g.lt(amin1, V(1.0));
  int f1 = 0, l1 = -1;
  V lat1 = V(0.0), obst1 = V(0.0);
  if (has_t1) {
    plan_grow(g, n1, amin1, TONGUE, f1, l1);
    lat1 = plan_max_lat(g, f1, l1);
  }
  // tongue constriction 2 (:1309-1392), kept when it does not touch the first
  bool has_t2 = false;
  int n2 = -1, l2 = -1;
  V lat2 = V(0.0), obst2 = V(0.0);
  if (has_t1) {
    V amin2;
    n2 = plan_argmin(g, TONGUE, amin2, f1, l1);
    if (g.lt(amin2, V(1.0))) {
      int f2;
      plan_grow(g, n2, amin2, TONGUE, f2, l2);
      if (f2 > l1 + 1 || l2 < f1 - 1) {
        has_t2 = true;
        lat2 = plan_max_lat(g, f2, l2);
      }
    }
  }
  // extent of the lip constriction (:1399-1444)
  const bool lip_c = g.lt(aminl, V(1.0));
  int ll = -1;
  if (lip_c) {
    int fl_;
    plan_grow(g, nl, aminl, LOWER_LIP, fl_, ll);
  }
  // positions of sections l1, l2 and ll + 1: Tube::calcPositions' sequential sum (:611-622)
  const int i1 = has_t1 ? l1 : -1, i2 = has_t2 ? l2 : -1, i3 = lip_c ? ll + 1 : -1;
  const int imax = i1 > i2 ? (i1 > i3 ? i1 : i3) : (i2 > i3 ? i2 : i3);
  V P1 = V(0.0), P2 = V(0.0), P3 = V(0.0);
  {
    V p = g.pos0();
    PLAN_LOOP
    for (int m = 0; m <= imax; ++m) {
      if (m == i1) P1 = p;
      if (m == i2) P2 = p;
      if (m == i3) P3 = p;
      p += g.len(m);
    }
  }
  // obstacles of the tongue constrictions (:1283-1299): the teeth when the jet ends within
  // 2 cm of them, else the middle of the section after the constriction
  V min_teeth = V(1000000.0);
  bool tb[2] = {false, false};
  auto tongue_obstacle = [&](const V &pl, int last, int narrow, bool &at_teeth) -> V {
    const V jet = pl + g.len(last);
    if (g.lt(teeth - jet, V(2.0))) {
      min_teeth = g.area(narrow);
      at_teeth = true;
      return teeth;
    }
    return (pl + g.len(last)) + 0.5 * g.len(last + 1);  // pos[last + 1] + 0.5 len[last + 1]
  };
  if (has_t1) obst1 = tongue_obstacle(P1, l1, n1, tb[0]);
  if (has_t2) obst2 = tongue_obstacle(P2, l2, n2, tb[1]);
  // the lower lip counts when narrower than a tongue constriction at the teeth
  const bool has_l = lip_c && g.lt(aminl, min_teeth);
  const V obstl = has_l ? P3 : V(0.0);

  // obstacle sections (:1456-1499)
  obst[0] = V(1.5);
  obst[1] = obst1;
  obst[2] = obst2;
  obst[3] = obstl;
  const bool has[4] = {true, has_t1, has_t2, has_l};
  uint32_t flags = 0;
  int mo[4] = {-1, -1, -1, -1};
  {  // the first section whose extent contains each obstacle (:1462-1471), one pass for all four
    V p = g.pos0();
    for (int c = 0; c < 4; ++c) po[c] = V(0.0);
    PLAN_LOOP
    for (int m = 0; m < NPM; ++m) {
      const V l = g.len(m);
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (has[c] && mo[c] < 0 && g.le(p, obst[c]) && g.le(obst[c], p + l)) {
          mo[c] = m;
          po[c] = p;
        }
      p += l;
      // (every constriction's section found: the rest of the scan changes nothing)
      if ((!has[1] || mo[1] >= 0) && (!has[2] || mo[2] >= 0) && (!has[3] || mo[3] >= 0) && mo[0] >= 0) break;
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (mo[c] >= 0) flags |= 1u << c;
  }
  if (g.lt(V(0.1), lat1)) flags |= PF_T1_LAT;
  if (g.lt(V(0.1), lat2)) flags |= PF_T2_LAT;
  if (g.lt(plan_abs(obst1 - teeth), V(0.0001))) flags |= PF_T1_TEETH;
  if (g.lt(plan_abs(obst2 - teeth), V(0.0001))) flags |= PF_T2_TEETH;
  key.n1 = n1; key.n2 = n2; key.nl = nl;
  key.l1 = l1; key.l2 = l2; key.ll = ll;
  for (int c = 0; c < 4; ++c) key.mo[c] = mo[c];
  key.has_t1 = has_t1; key.has_t2 = has_t2; key.lip_c = lip_c; key.has_l = has_l;
  key.tb1 = tb[0]; key.tb2 = tb[1];
  key.flags = flags;
}

// The words of a record that depend on the decisions alone: header and the outputs of the
// narrowest sections (an absent constriction points at section 25's).
AFS_HD inline void plan_key_words(const PlanKey &k, const SecRec *sec, uint64_t *w) {
  uint32_t up[4];
  for (int c = 0; c < 4; ++c) up[c] = k.mo[c] < 0 ? 0u : (uint32_t)k.mo[c];
  w[PW_HDR] = (uint64_t)k.flags | ((uint64_t)up[0] << 8) | ((uint64_t)up[1] << 16) | ((uint64_t)up[2] << 24) |
              ((uint64_t)up[3] << 32);
  const SecRec &q1 = sec[S_PHARYNX0 + (k.n1 < 0 ? 0 : k.n1)], &q2 = sec[S_PHARYNX0 + (k.n2 < 0 ? 0 : k.n2)];
  const SecRec &ql = sec[S_PHARYNX0 + (k.nl < 0 ? 0 : k.nl)];
  w[PW_UO] = (uint64_t)q1.x_uo0 | ((uint64_t)q1.x_uo1 << 16) | ((uint64_t)q2.x_uo0 << 32) | ((uint64_t)q2.x_uo1 << 48);
  w[PW_UOL] = (uint64_t)ql.x_uo0 | ((uint64_t)ql.x_uo1 << 16);
}

// The area terms of a narrowest section, A clamped to 0.1 cm^2 (:1502-1508): 1/A, sqrt(A) and
// 1/d = 1/sqrt(4A/pi).
AFS_HD inline void plan_area_terms(double a, double *t) {
#pragma clang fp contract(off)
  if (a < 0.1) a = 0.1;
  t[0] = 1.0 / a;
  t[1] = sqrt(a);
  t[2] = 1.0 / sqrt(4.0 * a / PI);
}

// The glottis dipole gain 0.5e-7 * 10^(aspiration dB / 20) (TdsModel.cpp:1546).
AFS_HD inline double plan_gain(double asp_db) { return 0.5e-7 * pow(10.0, asp_db / 20.0); }

// The plan of the sample at `ratio` between frames fl and fr.  sec: the kernel tables' section
// records (X_UN offsets of the section outputs).  two_mass: the glottis is the TwoMassModel,
// whose aspiration strength is Glottis::DEFAULT_ASPIRATION_STRENGTH_DB.
template <bool PRE = false>
AFS_HD inline void plan_sample(const afs_frame *fl, const afs_frame *fr, double ratio, const SecRec *sec,
                               bool two_mass, uint64_t *w) {
#pragma clang fp contract(off)
  const PlanGeomT<PRE> g{fl, fr, 1.0 - ratio, ratio};
  const double asp_db = two_mass ? GLOTTIS_DEFAULT_ASPIRATION_DB : g.r1 * fl->glottis[5] + ratio * fr->glottis[5];
  PlanKey k;
  double obst[4], po[4];
  plan_decide(g, k, obst, po);
  plan_key_words(k, sec, w);
  // downstream factors of the obstacle sections (:1472-1499)
  for (int c = 0; c < 4; ++c) w[PW_FDN + c] = plan_bits(k.mo[c] < 0 ? 0.0 : (obst[c] - po[c]) / g.len(k.mo[c]));
  const int na[3] = {k.n1, k.n2, k.nl};
  const int base[3] = {PW_T1, PW_T2, PW_L};
  for (int c = 0; c < 3; ++c) {
    double t[3];
    plan_area_terms(na[c] < 0 ? 1.0 : g.area(na[c]), t);
    w[base[c] + 0] = plan_bits(t[0]);
    w[base[c] + 1] = plan_bits(t[1]);
    if (c < 2) w[base[c] + 2] = plan_bits(t[2]);
  }
  w[PW_L + 2] = 0;
  w[PW_GAIN_G] = plan_bits(plan_gain(asp_db));
}

// ---------------------------------------------------------------------------
// Hop records (hops >= PLAN_HOP_MIN).  Within one hop (one frame transition) the decisions are
// almost always the same for every sample; the words then are functions of the ratio alone:
// the three area-term words of a narrowest section n are the terms of its interpolated area
// clampA((1-r) aL[n] + r aR[n]) (the same operations K5 and phase_interpolate perform), and a
// downstream factor (obstacle - position of its section) / length of its section is the ratio
// of two linear functions of r, whose values at the two frames K5 evaluates with the sample's
// formula on the frame alone.  A hop record carries, per word, its kind and up to four inputs;
// the synthesis kernel evaluates lane w's word at every sample (plan_word_eval).  A hop whose
// samples do not all share one PlanKey (or whose aspiration strength changes) is *mixed*: its
// samples keep the dense 128-B records.
// ---------------------------------------------------------------------------
enum : uint32_t { PK_CONST = 0, PK_INV = 1, PK_SQRT = 2, PK_INVD = 3, PK_FDN = 4 };
struct PlanHop {
  double p[PLAN_WORDS][4];  // lane w: its word's inputs (PK_CONST: the word's bits in p[w][0])
  uint8_t kind[PLAN_WORDS];
  uint32_t mixed;           // 1: the hop's samples use the dense records
  uint32_t dense;           // compact dense records (PlanArgs::compact): the mixed hop's slot
  uint64_t noise;           // plan_key_noise of every sample of the hop, or-ed (K1 picks its noise
                            // phases' variant for a launch from these, tree_kernel.h)
};
static_assert(sizeof(PlanHop) == 544, "hop record layout (K1 loads p[w] as two 16-byte words)");
constexpr int PLAN_HOP_MIN = 32;  // shorter hops (target sequences: hop 1) keep dense records

// Word w of the sample at `ratio` from its hop inputs, with the plan_sample operations (the
// synthesis kernel's branch-free form is tree_core.h plan_word_fast).
AFS_HD inline uint64_t plan_word_eval(uint32_t kind, const double *p, double ratio) {
#pragma clang fp contract(off)
  const double r1 = 1.0 - ratio;
  const double x = r1 * p[0] + ratio * p[1];
  const double y = r1 * p[2] + ratio * p[3];
  double t[3];
  plan_area_terms(plan_clampA(x), t);
  switch (kind) {
    case PK_INV: return plan_bits(t[0]);
    case PK_SQRT: return plan_bits(t[1]);
    case PK_INVD: return plan_bits(t[2]);
    case PK_FDN: return plan_bits(x / y);
    default: return plan_bits(p[0]);
  }
}

// Position of section m's start on the frame behind g (Tube::calcPositions' sequential sum).
template <bool PRE>
AFS_HD inline double plan_pos(const PlanGeomT<PRE> &g, int m) {
#pragma clang fp contract(off)
  double p = 0.0;
  for (int i = 0; i < m; ++i) p += g.len(i);
  return p;
}

// The inputs of a hop whose samples share the decisions k (fl, fr: the hop's frames).  Returns
// false when a word cannot be evaluated from them (the aspiration strength changes within the
// hop: the glottis gain is kept constant per hop).
AFS_HD inline bool plan_hop_inputs(const PlanKey &k, const afs_frame *fl, const afs_frame *fr, const SecRec *sec,
                                   bool two_mass, PlanHop &h) {
#pragma clang fp contract(off)
  uint64_t w[PLAN_WORDS];
  plan_key_words(k, sec, w);
  for (int q = 0; q < PLAN_WORDS; ++q) {
    h.kind[q] = PK_CONST;
    h.p[q][0] = plan_double(q < 3 ? w[q] : 0);
    h.p[q][1] = h.p[q][2] = h.p[q][3] = 0.0;
  }
  // downstream factors: (obstacle - position) and length at each frame
  const afs_frame *end[2] = {fl, fr};
  for (int e = 0; e < 2; ++e) {
    const PlanGeomT<false> g{end[e], end[e], 1.0, 0.0};  // the frame itself: 1 a + 0 a = a
    const double teeth = end[e]->teeth_position_cm;
    double obst[4] = {1.5, 0.0, 0.0, 0.0};
    const int last[2] = {k.l1, k.l2};
    const bool at_teeth[2] = {k.tb1, k.tb2};
    for (int c = 0; c < 2; ++c)
      if (k.mo[1 + c] >= 0)
        obst[1 + c] = at_teeth[c] ? teeth : (plan_pos(g, last[c]) + g.len(last[c])) + 0.5 * g.len(last[c] + 1);
    if (k.mo[3] >= 0) obst[3] = plan_pos(g, k.ll + 1);
    for (int c = 0; c < 4; ++c) {
      if (k.mo[c] < 0) continue;
      h.kind[PW_FDN + c] = PK_FDN;
      h.p[PW_FDN + c][e] = obst[c] - plan_pos(g, k.mo[c]);
      h.p[PW_FDN + c][2 + e] = g.len(k.mo[c]);
    }
  }
  // area terms of the narrowest sections
  const int na[3] = {k.n1, k.n2, k.nl};
  const int base[3] = {PW_T1, PW_T2, PW_L};
  for (int c = 0; c < 3; ++c) {
    const int nt = c < 2 ? 3 : 2;
    if (na[c] < 0) {
      double t[3];
      plan_area_terms(1.0, t);
      for (int j = 0; j < nt; ++j) h.p[base[c] + j][0] = t[j];
      continue;
    }
    for (int j = 0; j < nt; ++j) {
      h.kind[base[c] + j] = (uint8_t)(PK_INV + j);
      h.p[base[c] + j][0] = plan_clampA(fl->area_cm2[na[c]]);
      h.p[base[c] + j][1] = plan_clampA(fr->area_cm2[na[c]]);
    }
  }
  h.noise = plan_key_noise(k);
  // glottis gain: constant over the hop
  const double g0 = two_mass ? GLOTTIS_DEFAULT_ASPIRATION_DB : fl->glottis[5];
  h.p[PW_GAIN_G][0] = plan_gain(g0);
  return two_mass || fl->glottis[5] == fr->glottis[5];
}

// The decisions of every sample i0 .. i1-1 of the hop between fl and fr (ratios i / hop) with
// one evaluation on the interval geometry: true when every comparison was decided for all of
// them (k is then each sample's PlanKey), false when K5 has to decide the samples one by one.
template <bool PRE>
AFS_HD inline bool plan_hop_decide_iv(const afs_frame *fl, const afs_frame *fr, int hop, int i0, int i1, PlanKey &k) {
  const double rlo = (double)i0 / (double)hop, rhi = (double)(i1 - 1) / (double)hop;
  const PlanGeomIv<PRE> g{fl, fr, 1.0 - rlo, rlo, 1.0 - rhi, rhi, 0};
  PlanIv obst[4], po[4];
  plan_decide(g, k, obst, po);
  return g.undecided == 0;
}

// Host reference of K5's hop mode: the record of samples i0 .. i1-1 of the hop between fl and fr
// (ratios i / hop); the words of a mixed hop's samples come from plan_sample.
inline void plan_hop_host(const afs_frame *fl, const afs_frame *fr, int hop, int i0, int i1, const SecRec *sec,
                          bool two_mass, PlanHop &h) {
  uint64_t q0[2] = {0, 0}, noise = 0;
  PlanKey k0{};
  bool mixed = false;
  for (int i = i0; i < i1; ++i) {
    const double ratio = (double)i / (double)hop;
    const PlanGeomT<false> g{fl, fr, 1.0 - ratio, ratio};
    PlanKey k;
    double obst[4], po[4];
    plan_decide(g, k, obst, po);
    uint64_t q[2];
    plan_key_pack(k, q);
    noise |= plan_key_noise(k);
    if (i == i0) {
      k0 = k;
      q0[0] = q[0];
      q0[1] = q[1];
    } else if (q[0] != q0[0] || q[1] != q0[1]) {
      mixed = true;
    }
  }
  h = PlanHop{};
  if (!plan_hop_inputs(k0, fl, fr, sec, two_mass, h)) mixed = true;
  h.mixed = mixed ? 1u : 0u;
  h.noise = noise;
}

}  // namespace tree
}  // namespace afs
