// One Ed25519 verification per lane, ed25519-dalek 1.0.1 acceptance rules.
//
// Replaces, for one (pk, sig, msg) triple, the work behind
//   crypto::Signature::verify        (reference crypto/src/lib.rs:204-208)
//     -> ed25519::Signature::from_bytes, dalek::PublicKey::from_bytes,
//        PublicKey::verify_strict
//   crypto::Signature::verify_batch  (reference crypto/src/lib.rs:210-223)
//     -> per item: the same parse steps + the cofactorless equation
// and reports a flag byte (bit meanings in include/hsv.h):
//   S_OK      s < l                          (check_scalar)
//   A_OK      A decompresses                 (PublicKey::from_bytes)
//   R_OK      R decompresses                 (signature.R.decompress())
//   SMALL_A   A_OK and [8]A == O             (A.is_small_order())
//   SMALL_R   R_OK and [8]R == O             (signature_R.is_small_order())
//   PARSE_OK  S_OK and A_OK and R_OK
//   EQ_OK     PARSE_OK and [k](-A) + [s]B == R as points
//   STRICT_OK EQ_OK and not SMALL_A and not SMALL_R   (== verify_strict Ok)
//
// Work per lane (all lanes run the same instruction stream, no data-dependent
// branches):
//   SHA-512 of the single 96-byte block, Barrett reduction mod l,
//   decompress A (one x^((p-5)/8) chain), build [1..4](-A) (cached form),
//   signed WA-bit windows of k over ~253 doublings, with a signed WB-bit
//   window of s added from the LDS table of [1..2^(WB-1)]B every WB/WA windows,
//   decompress R and compare projectively.
#pragma once
#include "hsv_field.hpp"
#include "hsv_lattice.hpp"
#include "hsv_point.hpp"
#include "hsv_scalar.hpp"
#include "hsv_sha512.hpp"

namespace hsv {

enum : uint32_t {
  kStrictOk = 0x01,
  kEqOk = 0x02,
  kParseOk = 0x04,
  kSmallA = 0x08,
  kSmallR = 0x10,
  kSOk = 0x20,
  kAOk = 0x40,
  kROk = 0x80,
  // not a flag-byte bit: the device self-check failed for this item (see
  // fault_bit); kernels turn it into the launch's fault word and the host
  // into HSV_ERR_DEVICE_FAULT, never into a verdict
  kFault = 0x200,
};

// Fault injection modes (hsv_test_inject_fault; tests only): what the kernels
// read back in place of their table entries or workspace canary.
enum : uint32_t {
  kInjectNone = 0,
  kInjectZeroTables = 1,  // table entries read back as zeros
  kInjectCanary = 2,      // the lane's workspace canary is overwritten mid-batch
  kInjectFlipTables = 3,  // one bit of table entries flipped
  kInjectNoPublish = 4,   // fused transaction launch: record batch 0 is never published
};

// kFault when both points decoded (the equation is then part of the verdict)
// and the final accumulator q is not a curve point with Z != 0 (ge_is_sane).
HSV_INL uint32_t fault_bit(uint32_t a_ok, uint32_t r_ok, const ge_ext &q) {
  return (a_ok & r_ok & (ge_is_sane(q) ^ 1u)) ? (uint32_t)kFault : 0u;
}

// Shift a multi-limb value left by `sh` (0 < sh < 32) bits in place.
template <int N>
HSV_INL void limbs_shl(uint32_t x[N], int sh) {
  HSV_UNROLL
  for (int i = N - 1; i > 0; --i) x[i] = (x[i] << sh) | (x[i - 1] >> (32 - sh));
  x[0] <<= sh;
}

// Shift left by an arbitrary compile-time amount (0 <= SH < 32*N).
template <int N, int SH>
HSV_INL void limbs_shl_const(uint32_t x[N]) {
  constexpr int W = SH / 32, B = SH % 32;
  HSV_UNROLL
  for (int i = N - 1; i >= 0; --i) {
    uint32_t hi = (i - W >= 0) ? x[i - W] : 0u;
    uint32_t lo = (i - W - 1 >= 0) ? x[i - W - 1] : 0u;
    x[i] = B == 0 ? hi : ((hi << B) | (lo >> ((32 - B) & 31)));
  }
}

// Signed fixed-window recoding constant C_w = sum_{i<nwin} 2^(w-1) * 2^(w*i),
// limb j of it (compile-time).  Adding C_w to a scalar makes chunk i of the
// sum encode the digit chunk_i - 2^(w-1).
HSV_INL constexpr uint32_t recode_const_limb(int w, int nwin, int j) {
  uint32_t r = 0;
  for (int b = 0; b < 32; ++b) {
    const int bit = 32 * j + b;
    if (bit < w * nwin && bit % w == w - 1) r |= 1u << b;
  }
  return r;
}

template <int N, int W, int NWIN>
HSV_INL void recode_add(const uint32_t *x, int xlimbs, uint32_t out[N]) {
  uint64_t t = 0;
  HSV_UNROLL
  for (int j = 0; j < N; ++j) {
    t += (uint64_t)(j < xlimbs ? x[j] : 0u) + recode_const_limb(W, NWIN, j);
    out[j] = (uint32_t)t;
    t >>= 32;
  }
}

// Variable-base table [1..TS](-A), TS = 2^(WA-1), cached form.
template <int TS>
HSV_INL ge_cached select_cached(const ge_cached tab[TS], uint32_t chunk) {
  const int32_t d = (int32_t)chunk - TS;  // in [-TS, TS-1]
  const uint32_t neg = d < 0;
  const uint32_t mag = (uint32_t)(neg ? -d : d);
  ge_cached r = ge_cached_identity();
  HSV_UNROLL
  for (int m = 1; m <= TS; ++m) {
    const uint32_t take = (mag == (uint32_t)m);
    r.YpX = fe_select(r.YpX, tab[m - 1].YpX, take);
    r.YmX = fe_select(r.YmX, tab[m - 1].YmX, take);
    r.Z2 = fe_select(r.Z2, tab[m - 1].Z2, take);
    r.T2d = fe_select(r.T2d, tab[m - 1].T2d, take);
  }
  return ge_cached_cneg(r, neg);
}

// BTab must provide: ge_niels load(uint32_t idx) const  for idx in [0, 2^(WB-1))
// returning [idx+1]B.
template <int WB, class BTab>
HSV_INL ge_niels select_niels(const BTab &btab, uint32_t chunk) {
  const int32_t d = (int32_t)chunk - (1 << (WB - 1));
  const uint32_t neg = d < 0;
  const uint32_t mag = (uint32_t)(neg ? -d : d);
  const uint32_t idx = mag == 0 ? 0u : mag - 1u;
  ge_niels n = btab.load(idx);
  const uint32_t zero = (mag == 0);
  n.ypx = fe_select(n.ypx, fe_small(1), zero);
  n.ymx = fe_select(n.ymx, fe_small(1), zero);
  n.xy2d = fe_select(n.xy2d, fe_small(0), zero);
  return ge_niels_cneg(n, neg);
}

// tab[M-1] = [M]P for M = M0..TS, walking p = [M-1]P -> [M]P; recursion keeps
// every table index a compile-time constant (a runtime index would put the
// table in scratch memory).
template <int M, int TS>
HSV_INL void build_table_tail(ge_ext &p, ge_cached *tab) {
  if constexpr (M <= TS) {
    p = ge_add_cached<true>(p, tab[0]);
    tab[M - 1] = ge_to_cached(p);
    build_table_tail<M + 1, TS>(p, tab);
  }
}

// Window geometry.  WA: bits per variable-base (A) window; WB = M*WA bits per
// fixed-base (B) window, added every M-th A window.  NA windows cover the
// recoded k (k < 2^253 plus the recoding constant must stay below 2^(NA*WA)).
template <int WA, int WB>
struct Windows {
  static_assert(WB % WA == 0, "B windows must align with A windows");
  static constexpr int M = WB / WA;
  static constexpr int NA = (WA == 3) ? 85 : (256 / WA);   // 255 or 256 bits
  static constexpr int NB = (NA + M - 1) / M;
  static constexpr int TS = 1 << (WA - 1);                  // A table entries
  static constexpr int KBITS = NA * WA;                     // <= 256
  static constexpr int SBITS = NB * WB;                     // <= 288
  static_assert(KBITS <= 256 && SBITS <= 288, "window geometry");
};

// pk: 8 words, sig: 16 words (R = sig[0..7], s = sig[8..15]), msg: 8 words,
// all little-endian as loaded from memory.
template <int WA, int WB, class BTab>
HSV_INL uint32_t verify_one(const uint32_t pk[8], const uint32_t sig[16], const uint32_t msg[8],
                            const BTab &btab) {
  using G = Windows<WA, WB>;
  // --- s parse (check_scalar) -------------------------------------------
  const uint32_t s_ok = sc_is_canonical(sig + 8);

  // --- k = SHA-512(R || A || M) mod l  (original bytes, even if non-canonical)
  uint32_t h[16];
  sha512_96(sig, pk, msg, h);
  const sc k = sc_reduce512(h);

  // --- A = decompress(pk) ----------------------------------------------
  fe ax, ay;
  const uint32_t a_ok = ge_decompress(pk, ax, ay);
  const uint32_t small_a = a_ok & y_is_small_order(ay);

  // --- table [1..TS](-A) in cached form ----------------------------------
  ge_cached tab[G::TS];
  {
    ge_ext p1;
    p1.X = fe_carry(fe_neg(ax));
    p1.Y = ay;
    p1.Z = fe_small(1);
    p1.T = fe_mul(p1.X, ay);
    tab[0] = ge_to_cached(p1);
    if (G::TS >= 2) {
      ge_ext p2 = ge_dbl<true>(p1);
      tab[1] = ge_to_cached(p2);
      build_table_tail<3, G::TS>(p2, tab);  // 3P, 4P, ... (compile-time indices)
    }
  }

  // --- signed recodings, top window aligned to the top of the register ----
  uint32_t kr[8];
  recode_add<8, WA, G::NA>(k.v, 8, kr);
  limbs_shl_const<8, 256 - G::KBITS>(kr);
  uint32_t sr[9];
  recode_add<9, WB, G::NB>(sig + 8, 8, sr);
  limbs_shl_const<9, 288 - G::SBITS>(sr);

  // --- R' = [k](-A) + [s]B ---------------------------------------------
  ge_ext q = ge_identity();
  HSV_NOUNROLL
  for (int i = G::NA - 1; i >= 0; --i) {
    if (i != G::NA - 1) {
      HSV_UNROLL
      for (int j = 0; j < WA - 1; ++j) q = ge_dbl<false>(q);
      q = ge_dbl<true>(q);
    }
    const uint32_t ca = kr[7] >> (32 - WA);
    limbs_shl<8>(kr, WA);
    const ge_cached qa = select_cached<G::TS>(tab, ca);
    if (i % G::M == 0) {
      q = ge_add_cached<true>(q, qa);
      const uint32_t cb = sr[8] >> (32 - WB);
      limbs_shl<9>(sr, WB);
      const ge_niels nb = select_niels<WB>(btab, cb);
      q = ge_add_niels<false>(q, nb);
    } else {
      q = ge_add_cached<false>(q, qa);
    }
  }

  // --- R = decompress(sig.R), compare as points ------------------------
  fe rx, ry;
  const uint32_t r_ok = ge_decompress(sig, rx, ry);
  const uint32_t small_r = r_ok & y_is_small_order(ry);
  const uint32_t same = ge_eq_affine(q, rx, ry);

  const uint32_t parse_ok = s_ok & a_ok & r_ok;
  const uint32_t eq_ok = parse_ok & same;
  const uint32_t strict_ok = eq_ok & (small_a ^ 1u) & (small_r ^ 1u);
  return (strict_ok ? kStrictOk : 0u) | (eq_ok ? kEqOk : 0u) | (parse_ok ? kParseOk : 0u) |
         (small_a ? kSmallA : 0u) | (small_r ? kSmallR : 0u) | (s_ok ? kSOk : 0u) |
         (a_ok ? kAOk : 0u) | (r_ok ? kROk : 0u);
}

// ---------------------------------------------------------------------------
// Half-size-scalar verification (hsv_lattice.hpp).  With (c0, c1) from the
// lattice reduction of k (c0 == c1 k mod 8l, c1 odd) and b = (c1 s) mod l,
//   EQ_OK  <=>  [b]B + [c1](-R) + [|c0|](-sign(c0) A) == O.
// One Straus chain of NW windows of WA bits runs both variable bases (tables of
// [1..2^(WA-1)](-R) and of -sign(c0) A in registers) and the two fixed bases B
// and B' = [2^SPLIT]B (b = b_lo + 2^SPLIT b_hi, LDS tables, WB-bit windows).
// `fallback` is set when the reduction did not give short enough scalars; the
// caller then uses verify_one for that lane (flags are exact either way).
template <int WA, int WB>
struct HalfWindows {
  static_assert(WB % WA == 0, "B windows must align with A windows");
  static constexpr int M = WB / WA;
  static constexpr int NW = (WA == 3) ? 45 : (WA == 2 ? 68 : 34);  // 135 / 136 / 136 bits
  static constexpr int BITS = NW * WA;
  static constexpr int NBW = NW / M;
  // b_lo < 2^(BITS-2): b_lo + C_WB (about 0.502 * 2^BITS) must not carry out of BITS bits
  static constexpr int SPLIT = BITS - 2;
  static constexpr int TS = 1 << (WA - 1);
  static_assert(NW % M == 0 && NBW * WB == BITS, "window geometry");
  static_assert(BITS <= 160 && (kLatMaxBits + 2) <= BITS, "scalar bound vs loop length");
};

// x (5 limbs) + C_w over nwin windows, shifted so the top window sits at the top of 5 limbs
template <int W, int NWIN>
HSV_INL void recode_top5(const uint32_t x[5], uint32_t out[5]) {
  recode_add<5, W, NWIN>(x, 5, out);
  limbs_shl_const<5, 160 - W * NWIN>(out);
}

template <int WA, int WB, class BTab, class BTab2>
HSV_INL uint32_t verify_one_half(const uint32_t pk[8], const uint32_t sig[16], const uint32_t msg[8],
                                 const BTab &btab, const BTab2 &btab2, bool &fallback) {
  using G = HalfWindows<WA, WB>;
  const uint32_t s_ok = sc_is_canonical(sig + 8);
  uint32_t h[16];
  sha512_96(sig, pk, msg, h);
  const sc k = sc_reduce512(h);

  fe ax, ay, rx, ry;
  const uint32_t a_ok = ge_decompress(pk, ax, ay);
  const uint32_t small_a = a_ok & y_is_small_order(ay);
  const uint32_t r_ok = ge_decompress(sig, rx, ry);
  const uint32_t small_r = r_ok & y_is_small_order(ry);

  const LatOut lat = lattice_reduce(k);
  fallback = !lat.ok;
  const sc b = sc_mul_small(lat.c1, sig + 8);  // (c1 s) mod l

  // b = b_lo + 2^SPLIT b_hi
  uint32_t blo[5], bhi[5];
  HSV_UNROLL
  for (int i = 0; i < 5; ++i) {
    const int lo = 32 * i;
    blo[i] = lo + 32 <= G::SPLIT ? b.v[i] : (lo < G::SPLIT ? (b.v[i] & ((1u << (G::SPLIT - lo)) - 1u)) : 0u);
  }
  {
    constexpr int W = G::SPLIT / 32, S = G::SPLIT % 32;
    HSV_UNROLL
    for (int i = 0; i < 5; ++i) {
      const uint32_t x0 = (i + W < 8) ? b.v[i + W] : 0u;
      const uint32_t x1 = (i + W + 1 < 8) ? b.v[i + W + 1] : 0u;
      bhi[i] = S ? ((x0 >> S) | (x1 << ((32 - S) & 31))) : x0;
    }
  }

  // variable-base tables: [1..TS](-R) and [1..TS](-sign(c0) A)
  ge_cached tabr[G::TS], taba[G::TS];
  {
    ge_ext p1;
    p1.X = fe_carry(fe_neg(rx));
    p1.Y = ry;
    p1.Z = fe_small(1);
    p1.T = fe_mul(p1.X, p1.Y);
    tabr[0] = ge_to_cached(p1);
    if (G::TS >= 2) {
      ge_ext p2 = ge_dbl<true>(p1);
      tabr[1] = ge_to_cached(p2);
      build_table_tail<3, G::TS>(p2, tabr);
    }
  }
  {
    ge_ext p1;
    p1.X = fe_carry(fe_select(fe_neg(ax), ax, lat.c0_neg));
    p1.Y = ay;
    p1.Z = fe_small(1);
    p1.T = fe_mul(p1.X, p1.Y);
    taba[0] = ge_to_cached(p1);
    if (G::TS >= 2) {
      ge_ext p2 = ge_dbl<true>(p1);
      taba[1] = ge_to_cached(p2);
      build_table_tail<3, G::TS>(p2, taba);
    }
  }

  uint32_t dr[5], da[5], dlo[5], dhi[5];
  recode_top5<WA, G::NW>(lat.c1, dr);
  recode_top5<WA, G::NW>(lat.c0, da);
  recode_top5<WB, G::NBW>(blo, dlo);
  recode_top5<WB, G::NBW>(bhi, dhi);

  ge_ext q = ge_identity();
  HSV_NOUNROLL
  for (int i = G::NW - 1; i >= 0; --i) {
    if (i != G::NW - 1) {
      HSV_UNROLL
      for (int j = 0; j < WA - 1; ++j) q = ge_dbl<false>(q);
      q = ge_dbl<true>(q);
    }
    const uint32_t cr = dr[4] >> (32 - WA), ca = da[4] >> (32 - WA);
    limbs_shl<5>(dr, WA);
    limbs_shl<5>(da, WA);
    q = ge_add_cached<true>(q, select_cached<G::TS>(tabr, cr));
    if (i % G::M == 0) {
      q = ge_add_cached<true>(q, select_cached<G::TS>(taba, ca));
      const uint32_t cl = dlo[4] >> (32 - WB), ch = dhi[4] >> (32 - WB);
      limbs_shl<5>(dlo, WB);
      limbs_shl<5>(dhi, WB);
      q = ge_add_niels<true>(q, select_niels<WB>(btab, cl));
      q = ge_add_niels<false>(q, select_niels<WB>(btab2, ch));
    } else {
      q = ge_add_cached<false>(q, select_cached<G::TS>(taba, ca));
    }
  }
  // Q == O  <=>  X == 0 and Y == Z
  const uint32_t same = ge_is_neutral(q);

  const uint32_t parse_ok = s_ok & a_ok & r_ok;
  const uint32_t eq_ok = parse_ok & same;
  const uint32_t strict_ok = eq_ok & (small_a ^ 1u) & (small_r ^ 1u);
  return (strict_ok ? kStrictOk : 0u) | (eq_ok ? kEqOk : 0u) | (parse_ok ? kParseOk : 0u) |
         (small_a ? kSmallA : 0u) | (small_r ? kSmallR : 0u) | (s_ok ? kSOk : 0u) |
         (a_ok ? kAOk : 0u) | (r_ok ? kROk : 0u);
}


// ---------------------------------------------------------------------------
// Variable-base tables in memory.  Keeping [0..TS]P for two variable bases in
// VGPRs (2 x 5 x 40 registers) forces heavy spilling at two waves per SIMD,
// and a register-resident table is read with TS x 40 v_cndmask per addition.
// Instead each lane writes its tables once to a private region (VT) and reads
// one entry per addition by index: 8 x 16-byte loads issued a whole window
// (WA doublings) ahead of their use, no selects.  Entries are 4 field
// elements in the loose 256-bit encoding, 4 x 8 words = 128 bytes (one
// cache line).
//   VT::put(t, m, const uint32_t w[32])   store entry m of table t
//   VT::get(t, m, uint32_t w[32])         load it back
// Entry 0 is the identity, so a zero digit needs no special case.

// Entries use the loose 256-bit encoding (fe_pack_loose: one carry pass, no
// reduction below p); the limbs read back are class R.
HSV_INL void cached_pack(const ge_cached &c, uint32_t w[32]) {
  fe_pack_loose(c.YpX, w);
  fe_pack_loose(c.YmX, w + 8);
  fe_pack_loose(c.Z2, w + 16);
  fe_pack_loose(c.T2d, w + 24);
}

HSV_INL ge_cached cached_unpack(const uint32_t w[32]) {
  ge_cached c;
  c.YpX = fe_unpack_loose(w);
  c.YmX = fe_unpack_loose(w + 8);
  c.Z2 = fe_unpack_loose(w + 16);
  c.T2d = fe_unpack_loose(w + 24);
  return c;
}

// table t of VT <- [0..TS]P for the affine point (x, y)
template <int TS, class VT>
HSV_INL void vt_build(VT &vt, int t, const fe &x, const fe &y) {
#ifdef HSV_TIMING_STUB_TABLES  // tools/phase_probe.py only: tables left unwritten
  return;
#endif
  uint32_t w[32];
  cached_pack(ge_cached_identity(), w);
  vt.put(t, 0, w);
  ge_ext p1;
  p1.X = x;
  p1.Y = y;
  p1.Z = fe_small(1);
  p1.T = fe_mul(x, y);
  const ge_cached c1 = ge_to_cached(p1);
  cached_pack(c1, w);
  vt.put(t, 1, w);
  if (TS >= 2) {
    // [m]P = [m-1]P + P with P as an affine Niels point (Z = 1: the mixed
    // addition is one multiply cheaper than the cached one)
    ge_niels n1;
    n1.ypx = fe_add(y, x);
    n1.ymx = fe_sub(y, x);
    n1.xy2d = fe_mul(p1.T, fe_d2());
    ge_ext p = ge_dbl<true>(p1);
    cached_pack(ge_to_cached(p), w);
    vt.put(t, 2, w);
    HSV_NOUNROLL
    for (int m = 3; m <= TS; ++m) {
      p = ge_add_niels<true>(p, n1);
      cached_pack(ge_to_cached(p), w);
      vt.put(t, m, w);
    }
  }
}

// signed digit (chunk - TS) -> table index |d| and sign
template <int TS>
HSV_INL uint32_t digit_mag(uint32_t chunk, uint32_t &neg) {
  const int32_t d = (int32_t)chunk - TS;
  neg = d < 0;
  return (uint32_t)(d < 0 ? -d : d);
}

// Full-length verification with the table of -A in VT (table 0): the
// fallback of the half-size path for the rare lanes without short scalars.
template <int WA, int WB, class BTab, class VT>
HSV_INL uint32_t verify_one_mt(const uint32_t pk[8], const uint32_t sig[16], const uint32_t msg[8],
                               const BTab &btab, VT &vt) {
  using G = Windows<WA, WB>;
  const uint32_t s_ok = sc_is_canonical(sig + 8);
  uint32_t h[16];
  sha512_96(sig, pk, msg, h);
  const sc k = sc_reduce512(h);
  fe ax, ay;
  const uint32_t a_ok = ge_decompress(pk, ax, ay);
  const uint32_t small_a = a_ok & y_is_small_order(ay);
  vt_build<G::TS>(vt, 0, fe_carry(fe_neg(ax)), ay);

  uint32_t kr[8];
  recode_add<8, WA, G::NA>(k.v, 8, kr);
  limbs_shl_const<8, 256 - G::KBITS>(kr);
  uint32_t sr[9];
  recode_add<9, WB, G::NB>(sig + 8, 8, sr);
  limbs_shl_const<9, 288 - G::SBITS>(sr);

  ge_ext q = ge_identity();
  HSV_NOUNROLL
  for (int i = G::NA - 1; i >= 0; --i) {
    uint32_t na;
    const uint32_t ma = digit_mag<G::TS>(kr[7] >> (32 - WA), na);
    limbs_shl<8>(kr, WA);
    uint32_t wa[32];
    vt.get(0, ma, wa);
    if (i != G::NA - 1) {
      HSV_UNROLL
      for (int j = 0; j < WA - 1; ++j) q = ge_dbl<false>(q);
      q = ge_dbl<true>(q);
    }
    const ge_cached qa = ge_cached_cneg(cached_unpack(wa), na);
    if (i % G::M == 0) {
      q = ge_add_cached<true>(q, qa);
      const uint32_t cb = sr[8] >> (32 - WB);
      limbs_shl<9>(sr, WB);
      q = ge_add_niels<false>(q, select_niels<WB>(btab, cb));
    } else {
      q = ge_add_cached<false>(q, qa);
    }
  }
  fe rx, ry;
  const uint32_t r_ok = ge_decompress(sig, rx, ry);
  const uint32_t small_r = r_ok & y_is_small_order(ry);
  const uint32_t same = ge_eq_affine(q, rx, ry);
  const uint32_t parse_ok = s_ok & a_ok & r_ok;
  const uint32_t eq_ok = parse_ok & same;
  const uint32_t strict_ok = eq_ok & (small_a ^ 1u) & (small_r ^ 1u);
  return (strict_ok ? kStrictOk : 0u) | (eq_ok ? kEqOk : 0u) | (parse_ok ? kParseOk : 0u) |
         (small_a ? kSmallA : 0u) | (small_r ? kSmallR : 0u) | (s_ok ? kSOk : 0u) |
         (a_ok ? kAOk : 0u) | (r_ok ? kROk : 0u);
}

// Half-size-scalar verification (same equation as verify_one_half) with the
// tables of -R (table 0) and -sign(c0) A (table 1) in VT.
template <int WA, int WB, class BTab, class BTab2, class VT>
HSV_INL uint32_t verify_one_half_mt(const uint32_t pk[8], const uint32_t sig[16], const uint32_t msg[8],
                                    const BTab &btab, const BTab2 &btab2, VT &vt, bool &fallback) {
  using G = HalfWindows<WA, WB>;
  const uint32_t s_ok = sc_is_canonical(sig + 8);
  uint32_t h[16];
  sha512_96(sig, pk, msg, h);
  const sc k = sc_reduce512(h);

  const LatOut lat = lattice_reduce(k);
  fallback = !lat.ok;

  uint32_t a_ok, small_a, r_ok, small_r;
  {
    fe x, y;
    r_ok = ge_decompress(sig, x, y);
    small_r = r_ok & y_is_small_order(y);
    vt_build<G::TS>(vt, 0, fe_carry(fe_neg(x)), y);
  }
  {
    fe x, y;
    a_ok = ge_decompress(pk, x, y);
    small_a = a_ok & y_is_small_order(y);
    vt_build<G::TS>(vt, 1, fe_carry(fe_select(fe_neg(x), x, lat.c0_neg)), y);
  }

  uint32_t dr[5], da[5], dlo[5], dhi[5];
  {
    const sc b = sc_mul_small(lat.c1, sig + 8);  // (c1 s) mod l = b_lo + 2^SPLIT b_hi
    uint32_t blo[5], bhi[5];
    HSV_UNROLL
    for (int i = 0; i < 5; ++i) {
      const int lo = 32 * i;
      blo[i] = lo + 32 <= G::SPLIT ? b.v[i] : (lo < G::SPLIT ? (b.v[i] & ((1u << (G::SPLIT - lo)) - 1u)) : 0u);
    }
    constexpr int W = G::SPLIT / 32, S = G::SPLIT % 32;
    HSV_UNROLL
    for (int i = 0; i < 5; ++i) {
      const uint32_t x0 = (i + W < 8) ? b.v[i + W] : 0u;
      const uint32_t x1 = (i + W + 1 < 8) ? b.v[i + W + 1] : 0u;
      bhi[i] = S ? ((x0 >> S) | (x1 << ((32 - S) & 31))) : x0;
    }
    recode_top5<WA, G::NW>(lat.c1, dr);
    recode_top5<WA, G::NW>(lat.c0, da);
    recode_top5<WB, G::NBW>(blo, dlo);
    recode_top5<WB, G::NBW>(bhi, dhi);
  }

  ge_ext q = ge_identity();
  HSV_NOUNROLL
  for (int i = G::NW - 1; i >= 0; --i) {
    uint32_t nr, na;
    const uint32_t mr = digit_mag<G::TS>(dr[4] >> (32 - WA), nr);
    const uint32_t ma = digit_mag<G::TS>(da[4] >> (32 - WA), na);
    limbs_shl<5>(dr, WA);
    limbs_shl<5>(da, WA);
    uint32_t wr[32], wa[32];
    vt.get(0, mr, wr);  // in flight during the doublings
    vt.get(1, ma, wa);
    if (i != G::NW - 1) {
      HSV_UNROLL
      for (int j = 0; j < WA - 1; ++j) q = ge_dbl<false>(q);
      q = ge_dbl<true>(q);
    }
    q = ge_add_cached<true>(q, ge_cached_cneg(cached_unpack(wr), nr));
    const ge_cached qa = ge_cached_cneg(cached_unpack(wa), na);
    if (i % G::M == 0) {
      q = ge_add_cached<true>(q, qa);
      const uint32_t cl = dlo[4] >> (32 - WB), ch = dhi[4] >> (32 - WB);
      limbs_shl<5>(dlo, WB);
      limbs_shl<5>(dhi, WB);
      q = ge_add_niels<true>(q, select_niels<WB>(btab, cl));
      q = ge_add_niels<false>(q, select_niels<WB>(btab2, ch));
    } else {
      q = ge_add_cached<false>(q, qa);
    }
  }
  const uint32_t same = ge_is_neutral(q);  // Q == O

  const uint32_t parse_ok = s_ok & a_ok & r_ok;
  const uint32_t eq_ok = parse_ok & same;
  const uint32_t strict_ok = eq_ok & (small_a ^ 1u) & (small_r ^ 1u);
  return (strict_ok ? kStrictOk : 0u) | (eq_ok ? kEqOk : 0u) | (parse_ok ? kParseOk : 0u) |
         (small_a ? kSmallA : 0u) | (small_r ? kSmallR : 0u) | (s_ok ? kSOk : 0u) |
         (a_ok ? kAOk : 0u) | (r_ok ? kROk : 0u);
}

}  // namespace hsv
