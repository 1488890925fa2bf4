#pragma once
// kron.hpp -- the Graph500 Kronecker edge stream the reference uses for its R-MAT inputs, as
// host/device inline functions (shared by the device generator kron.hip and the host build rmat.cpp).
//
// Reference semantics (packed path, DistEdgeList::GenGraph500Data(packed=true),
// include/CombBLAS/DistEdgeList.cpp:223-237 -> RefGen21::make_graph, RefGen21.h:285-303):
//   * seed: userseed = SEED env or 0xDECAFBAD (RefGen21.h:306-318); five MRG seed words
//     (make_mrg_seed(userseed, userseed), graph500-1.2/generator/utils.c);
//   * scramble constants val0/val1: the seeded state skipped by 50*2^128 + 7*2^64 steps, two pairs of
//     draws combined as x*0xFFFFFFFF + y (MakeScrambleValues, RefGen21.h:226-240);
//   * edge ei: the seeded state skipped by ei*2^64 steps (generate_kronecker_range, RefGen21.h:246-262),
//     then one 4-way Bernoulli draw per level with rejection below 0xFFFFFFFF % 10000 and the
//     quadrant order b, c, a, d (generate_4way_bernoulli, RefGen21.h:100-130), clip-and-flip while
//     src == tgt (make_one_edge, RefGen21.h:196-222), and the bit-reverse scramble of both ends
//     (scramble, RefGen21.h:183-194).
// The random number generator is L'Ecuyer's order-5 MRG modulo 2^31-1 (x = 107374182, y = 104480;
// graph500-1.2/generator/splittable_mrg.c).  A transition A^n is fully described by the bottom row
// (s, t, u, v, w) of its matrix (the rest follows from x and y); jumps use A^(k*256^i) tables built
// here by repeated squaring (the reference ships the same powers precomputed in mrg_transitions.c).
#include <stdint.h>

#if defined(__HIPCC__)
#define CBG_KHD __host__ __device__ __forceinline__
#else
#define CBG_KHD inline
#endif

namespace cbg { namespace kron {

constexpr uint32_t kP = 0x7FFFFFFFu;   // 2^31 - 1
constexpr uint32_t kX = 107374182u, kY = 104480u;
constexpr uint64_t kDefaultSeed = 0xDECAFBADull;
constexpr int kSkipBytes = 5;          // edge indices < 2^40 (scale <= 35 at edge factor 16)

CBG_KHD uint32_t mred(uint64_t t) {    // t < 2^62 -> t mod p
  uint32_t r = (uint32_t)(t & kP) + (uint32_t)(t >> 31);
  return r >= kP ? r - kP : r;
}
CBG_KHD uint32_t madd(uint32_t a, uint32_t b) { uint32_t r = a + b; return r >= kP ? r - kP : r; }
CBG_KHD uint32_t mmul(uint32_t a, uint32_t b) { return mred((uint64_t)a * b); }

struct Mat {                  // bottom row of A^n plus the derived column a..d (a = x s + t, ...)
  uint32_t s, t, u, v, w, a, b, c, d;
};
struct State { uint32_t z1, z2, z3, z4, z5; };

CBG_KHD void fill(Mat& m) {
  m.a = madd(mmul(m.s, kX), m.t);
  m.b = madd(mmul(m.a, kX), m.u);
  m.c = madd(mmul(m.b, kX), m.v);
  m.d = madd(mmul(m.c, kX), m.w);
}
CBG_KHD Mat identity() { Mat m{0, 0, 0, 0, 1, 0, 0, 0, 0}; fill(m); return m; }
CBG_KHD Mat step_matrix() { Mat m{0, 0, 0, 1, 0, 0, 0, 0, 0}; fill(m); return m; }

// sum of products mod p, each product < 2^62: accumulate with one reduction per term
CBG_KHD uint32_t dot(uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1, uint32_t a2, uint32_t b2,
                     uint32_t a3, uint32_t b3, uint32_t a4, uint32_t b4) {
  uint32_t r = mmul(a0, b0);
  r = mred((uint64_t)a1 * b1 + r);
  r = mred((uint64_t)a2 * b2 + r);
  r = mred((uint64_t)a3 * b3 + r);
  return mred((uint64_t)a4 * b4 + r);
}

// Full 5x5 matrix of A^n in row-major order:
//   [d  sy ay by cy]
//   [c  w  sy ay by]
//   [b  v  w  sy ay]
//   [a  u  v  w  sy]
//   [s  t  u  v  w ]
CBG_KHD void expand(const Mat& m, uint32_t M[5][5]) {
  const uint32_t sy = mmul(m.s, kY), ay = mmul(m.a, kY), by = mmul(m.b, kY), cy = mmul(m.c, kY);
  const uint32_t r0[5] = {m.d, sy, ay, by, cy};
  const uint32_t r1[5] = {m.c, m.w, sy, ay, by};
  const uint32_t r2[5] = {m.b, m.v, m.w, sy, ay};
  const uint32_t r3[5] = {m.a, m.u, m.v, m.w, sy};
  const uint32_t r4[5] = {m.s, m.t, m.u, m.v, m.w};
  for (int j = 0; j < 5; ++j) { M[0][j] = r0[j]; M[1][j] = r1[j]; M[2][j] = r2[j]; M[3][j] = r3[j]; M[4][j] = r4[j]; }
}

// state <- A^n state  (state as the column (z1..z5))
CBG_KHD void apply(const Mat& m, State& z) {
  uint32_t M[5][5];
  expand(m, M);
  const uint32_t in[5] = {z.z1, z.z2, z.z3, z.z4, z.z5};
  uint32_t o[5];
  for (int i = 0; i < 5; ++i) o[i] = dot(M[i][0], in[0], M[i][1], in[1], M[i][2], in[2], M[i][3], in[3], M[i][4], in[4]);
  z.z1 = o[0]; z.z2 = o[1]; z.z3 = o[2]; z.z4 = o[3]; z.z5 = o[4];
}

// product of two powers of A (they commute): the bottom row of M*N
CBG_KHD Mat mul(const Mat& m, const Mat& n) {
  uint32_t M[5][5], N[5][5];
  expand(m, M);
  expand(n, N);
  Mat r;
  uint32_t row[5];
  for (int j = 0; j < 5; ++j) row[j] = dot(M[4][0], N[0][j], M[4][1], N[1][j], M[4][2], N[2][j], M[4][3], N[3][j], M[4][4], N[4][j]);
  r.s = row[0]; r.t = row[1]; r.u = row[2]; r.v = row[3]; r.w = row[4];
  fill(r);
  return r;
}

CBG_KHD Mat power(Mat m, uint64_t e) {
  Mat r = identity();
  while (e) {
    if (e & 1) r = mul(r, m);
    m = mul(m, m);
    e >>= 1;
  }
  return r;
}

// one step with the original generator: z1' = x z1 + y z5, the rest shift down; returns z1'
CBG_KHD uint32_t next(State& z) {
  const uint32_t n = mred((uint64_t)kX * z.z1 + mmul(kY, z.z5));
  z.z5 = z.z4; z.z4 = z.z3; z.z3 = z.z2; z.z2 = z.z1; z.z1 = n;
  return n;
}

CBG_KHD State seed_state(uint64_t userseed) {   // make_mrg_seed(userseed, userseed)
  State z;
  z.z1 = (uint32_t)((userseed & 0x3FFFFFFF) + 1);
  z.z2 = (uint32_t)(((userseed >> 30) & 0x3FFFFFFF) + 1);
  z.z3 = (uint32_t)((userseed & 0x3FFFFFFF) + 1);
  z.z4 = (uint32_t)(((userseed >> 30) & 0x3FFFFFFF) + 1);
  z.z5 = (uint32_t)(((userseed >> 60) << 4) + (userseed >> 60) + 1);
  return z;
}

CBG_KHD uint64_t bitrev64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_bitreverse64(x);
#else
  x = __builtin_bswap64(x);
  x = ((x >> 4) & 0x0F0F0F0F0F0F0F0Full) | ((x & 0x0F0F0F0F0F0F0F0Full) << 4);
  x = ((x >> 2) & 0x3333333333333333ull) | ((x & 0x3333333333333333ull) << 2);
  x = ((x >> 1) & 0x5555555555555555ull) | ((x & 0x5555555555555555ull) << 1);
  return x;
#endif
}

CBG_KHD int64_t scramble(int64_t v0, int lgN, uint64_t val0, uint64_t val1) {
  uint64_t v = (uint64_t)v0;
  v += val0 + val1;
  v *= (val0 | 0x4519840211493211ull);
  v = bitrev64(v) >> (64 - lgN);
  v *= (val1 | 0x3050852102C843A5ull);
  v = bitrev64(v) >> (64 - lgN);
  return (int64_t)v;
}

// quadrant of one level: 1 = b, 2 = c, 0 = a, 3 = d (initiator .57/.19/.19/.05 in 1/10000 units)
CBG_KHD int quadrant(State& z) {
  const uint32_t limit = 0xFFFFFFFFu % 10000u;
  uint32_t val = next(z);
  while (val < limit) val = next(z);
  val %= 10000u;
  if (val < 1900u) return 1;
  val -= 1900u;
  if (val < 1900u) return 2;
  val -= 1900u;
  if (val < 5700u) return 0;
  return 3;
}

// edge from a state already skipped to the edge's position: (src, tgt) before scrambling
CBG_KHD void edge_unscrambled(State z, int lgN, int64_t* src, int64_t* tgt) {
  int64_t nv = (int64_t)1 << lgN, bs = 0, bt = 0;
  while (nv > 1) {
    const int sq = quadrant(z);
    int so = sq / 2, to = sq % 2;
    if (bs == bt && so > to) { const int t = so; so = to; to = t; }
    nv /= 2;
    bs += nv * so;
    bt += nv * to;
  }
  *src = bs;
  *tgt = bt;
}

// Skip tables: tab[i*256 + k] = A^(k * 256^(8+i) )  (i < kSkipBytes), i.e. the jumps of the edge index
// bytes (the reference's exponent_middle, bytes 8.. of the 192-bit exponent).
struct Params {
  State base;            // seeded state
  uint64_t val0, val1;   // scramble constants
};

inline Params make_params(uint64_t userseed, Mat* tab /* kSkipBytes*256 entries */) {
  Mat b64 = power(step_matrix(), 1ull << 32);       // A^(2^64) = (A^(2^32))^(2^32)
  b64 = power(b64, 1ull << 32);
  Mat byte = b64;                                   // A^(256^(8+i))
  for (int i = 0; i < kSkipBytes; ++i) {
    tab[i * 256] = identity();
    tab[i * 256 + 1] = byte;
    for (int k = 2; k < 256; ++k) tab[i * 256 + k] = mul(tab[i * 256 + k - 1], byte);
    byte = power(byte, 256);
  }
  Params p;
  p.base = seed_state(userseed);
  // MakeScrambleValues: skip(high = 50, middle = 7, low = 0) = A^(50 * 2^128 + 7 * 2^64)
  State z = p.base;
  const Mat b128 = power(b64, 1ull << 32);
  apply(power(power(b128, 1ull << 32), 50), z);     // (A^(2^64))^(2^64) = A^(2^128)
  apply(tab[7], z);
  uint64_t v0 = next(z);
  v0 *= 0xFFFFFFFFull;
  v0 += next(z);
  uint64_t v1 = next(z);
  v1 *= 0xFFFFFFFFull;
  v1 += next(z);
  p.val0 = v0;
  p.val1 = v1;
  return p;
}

// the scrambled edge ei
CBG_KHD void edge(const Params& p, const Mat* tab, int lgN, uint64_t ei, int64_t* src, int64_t* tgt) {
  State z = p.base;
  for (int i = 0; ei; ++i, ei >>= 8) {
    const uint32_t k = (uint32_t)(ei & 0xFF);
    if (k) apply(tab[i * 256 + k], z);
  }
  int64_t s, t;
  edge_unscrambled(z, lgN, &s, &t);
  *src = scramble(s, lgN, p.val0, p.val1);
  *tgt = scramble(t, lgN, p.val0, p.val1);
}

}  // namespace kron
}  // namespace cbg
