// pyset.h — CPython 3.10 hash / set-iteration-order emulation, host and device.
//
// Why this exists: the reference picks a clique's consensus box with
//   max(subgraph.degree(weight="weight"), key=lambda x: x[1])[0]      (get_cliques.py:182-183)
// and `max` keeps the FIRST maximal element.  The subgraph's node iteration order is the
// iteration order of the CPython set `set(tuple(sorted(clique)))` built by networkx
// (graph.py Graph.subgraph -> filters.py show_nodes -> coreviews.py FilterAtlas.__iter__),
// i.e. it depends on CPython's hash of the (x: float, y: float, id: int) node keys and on
// the set's open-addressing probe sequence.  When degrees tie (about 1 % of cliques on
// EMPIAR-10017, far more with duplicate boxes) the consensus box is decided here.
//
// Restated from the published CPython 3.10 algorithms (Python/pyhash.c _Py_HashDouble,
// Objects/longobject.c long_hash, Objects/tupleobject.c tuplehash (xxHash-based),
// Objects/setobject.c set_add_entry / set_table_resize / set_insert_clean; PySet_MINSIZE 8,
// LINEAR_PROBES 9, PERTURB_SHIFT 5).  Validated against the live interpreter by
// tests/test_pyset.py.
#pragma once
#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#define PYS_FN __host__ __device__ __forceinline__
#else
#define PYS_FN static inline
#endif

namespace pyset {

constexpr int HASH_BITS = 61;
constexpr uint64_t HASH_MOD = (1ULL << HASH_BITS) - 1;
constexpr uint64_t HASH_INF = 314159ULL;

// _Py_HashDouble for finite / infinite values (NaN never reaches a graph node).
PYS_FN uint64_t hash_double(double v) {
  if (!isfinite(v)) {
    if (isinf(v)) return v > 0 ? HASH_INF : (uint64_t)(-(int64_t)HASH_INF);
    return 0;  // unreachable for graph nodes (NaN coordinates never form edges)
  }
  // integral values below 2^53 (integer pixel coordinates): CPython guarantees
  // hash(x) == hash(int(x)), i.e. sign * (|x| mod P) with |x| < P, -1 -> -2; this skips the
  // frexp / 28-bit mantissa loop for them (same result as the loop below)
  if (fabs(v) < 9007199254740992.0 && v == trunc(v)) {
    uint64_t x = (uint64_t)(int64_t)v;
    if (x == (uint64_t)-1) x = (uint64_t)-2;
    return x;
  }
  int e;
  double m = frexp(v, &e);
  int sign = 1;
  if (m < 0) { sign = -1; m = -m; }
  uint64_t x = 0;
  while (m != 0.0) {
    x = ((x << 28) & HASH_MOD) | x >> (HASH_BITS - 28);
    m *= 268435456.0;  // 2**28
    e -= 28;
    uint64_t y = (uint64_t)m;
    m -= (double)y;
    x += y;
    if (x >= HASH_MOD) x -= HASH_MOD;
  }
  e = e >= 0 ? e % HASH_BITS : HASH_BITS - 1 - ((-1 - e) % HASH_BITS);
  x = ((x << e) & HASH_MOD) | x >> (HASH_BITS - e);
  x = x * (uint64_t)(int64_t)sign;
  if (x == (uint64_t)-1) x = (uint64_t)-2;
  return x;
}

// long_hash for a non-negative id.
PYS_FN uint64_t hash_id(int64_t v) {
  uint64_t x = (uint64_t)v < HASH_MOD ? (uint64_t)v : (uint64_t)v % HASH_MOD;
  if (x == (uint64_t)-1) x = (uint64_t)-2;
  return x;
}

constexpr uint64_t XXPRIME_1 = 11400714785074694791ULL;
constexpr uint64_t XXPRIME_2 = 14029467366897019727ULL;
constexpr uint64_t XXPRIME_5 = 2870177450012600261ULL;

// The multipliers as scalar-register values made inside the caller's loop: left as plain
// literals, the compiler hoists them into vector registers for the whole fused kernel, where
// they were spilled to scratch (rgc_fused.hip's order pass runs them rarely).
#if defined(__HIP_DEVICE_COMPILE__)
template <uint64_t C>
__device__ __forceinline__ uint64_t pys_sconst() {
  uint32_t lo, hi;
  asm volatile("s_mov_b32 %0, %1" : "=s"(lo) : "i"((uint32_t)(C & 0xFFFFFFFFu)));
  asm volatile("s_mov_b32 %0, %1" : "=s"(hi) : "i"((uint32_t)(C >> 32)));
  return ((uint64_t)hi << 32) | lo;
}
#define PYS_CONST(C) pys_sconst<C>()
#else
#define PYS_CONST(C) (C)
#endif

PYS_FN uint64_t xx_round(uint64_t acc, uint64_t lane) {
  acc += lane * PYS_CONST(XXPRIME_2);
  acc = (acc << 31) | (acc >> 33);
  acc *= PYS_CONST(XXPRIME_1);
  return acc;
}

// hash((x, y, id)) — the networkx node key built by add_nodes_to_graph (get_cliques.py:33-34).
PYS_FN uint64_t hash_node(double x, double y, int64_t id) {
  uint64_t acc = PYS_CONST(XXPRIME_5);
  acc = xx_round(acc, hash_double(x));
  acc = xx_round(acc, hash_double(y));
  acc = xx_round(acc, hash_id(id));
  acc += PYS_CONST(3ULL ^ (XXPRIME_5 ^ 3527539ULL));
  if (acc == (uint64_t)-1) return 1546275796ULL;
  return acc;
}

// Probe for a free slot exactly like set_add_entry / set_insert_clean with no dummies and
// no equal keys (all node keys of a clique are distinct).
PYS_FN int probe_free(const int8_t* slot, uint64_t mask, uint64_t hash) {
  uint64_t perturb = hash;
  uint64_t i = hash & mask;
  while (true) {
    if (slot[i] < 0) return (int)i;
    if (i + 9 <= mask) {
      for (int j = 1; j <= 9; ++j)
        if (slot[i + j] < 0) return (int)(i + j);
    }
    perturb >>= 5;
    i = (i * 5 + 1 + perturb) & mask;
  }
}

// Iteration order of `set(keys)` where keys are inserted in the given order (n <= 18).
// hashes[t] is the hash of the t-th inserted key; out[r] = insertion index of the r-th key
// yielded by iteration.  Returns n.
PYS_FN int set_order(const uint64_t* hashes, int n, int8_t* out) {
  int8_t tab[32];
  uint64_t mask = 7;
  for (int i = 0; i < 32; ++i) tab[i] = -1;
  int fill = 0;
  for (int t = 0; t < n; ++t) {
    int s = probe_free(tab, mask, hashes[t]);
    tab[s] = (int8_t)t;
    ++fill;
    if (!((uint64_t)fill * 5 < mask * 3)) {
      // set_table_resize(so, used*4): smallest power of two > used*4, >= 8
      uint64_t minused = (uint64_t)fill * 4, newsize = 8;
      while (newsize <= minused) newsize <<= 1;
      int8_t old[32];
      uint64_t oldmask = mask;
      for (int i = 0; i < 32; ++i) { old[i] = tab[i]; tab[i] = -1; }
      mask = newsize - 1;
      for (uint64_t i = 0; i <= oldmask; ++i)
        if (old[i] >= 0) tab[probe_free(tab, mask, hashes[old[i]])] = old[i];
    }
  }
  int r = 0;
  for (uint64_t i = 0; i <= mask; ++i)
    if (tab[i] >= 0) out[r++] = tab[i];
  return r;
}

// ---- register-resident variant for the device epilogue (no stack arrays, so no scratch):
// the 32-slot table lives in two u64 words as 4-bit slots (15 = empty), keys n <= 8 (a set of
// <= 8 keys never grows past 32 slots: one resize at fill 5 -> 32).
PYS_FN int pk_get(uint64_t lo, uint64_t hi, uint64_t i) {
  return (int)(((i < 16 ? lo : hi) >> (4 * (i & 15))) & 15);
}
PYS_FN void pk_set(uint64_t& lo, uint64_t& hi, uint64_t i, int v) {
  const uint64_t sh = 4 * (i & 15);
  const uint64_t m = ~(15ULL << sh), b = (uint64_t)v << sh;
  if (i < 16) lo = (lo & m) | b; else hi = (hi & m) | b;
}
PYS_FN uint64_t pk_probe(uint64_t lo, uint64_t hi, uint64_t mask, uint64_t hash) {
  uint64_t perturb = hash;
  uint64_t i = hash & mask;
  while (true) {
    if (pk_get(lo, hi, i) == 15) return i;
    if (i + 9 <= mask) {
      for (uint64_t j = 1; j <= 9; ++j)
        if (pk_get(lo, hi, i + j) == 15) return i + j;
    }
    perturb >>= 5;
    i = (i * 5 + 1 + perturb) & mask;
  }
}
// Same result as set_order for N <= 8 keys, packed: nibble r = insertion index of the r-th
// key yielded by iteration.  Every private array is indexed at compile time: the one resize a
// set of <= 8 keys goes through (fill 5: 8 -> 32 slots) re-inserts the five keys in old-slot
// order through a compare-exchange network instead of a table lookup.
template <int N>
PYS_FN uint32_t set_order_packed(const uint64_t (&h)[N]) {
  static_assert(N >= 1 && N <= 8, "packed set order supports 1..8 keys");
  uint64_t lo = ~0ULL, hi = ~0ULL, mask = 7;
  uint64_t slot[N];
#pragma unroll
  for (int t = 0; t < N; ++t) {
    slot[t] = pk_probe(lo, hi, mask, h[t]);
    pk_set(lo, hi, slot[t], t);
    if (N > 4 && t == 4) {   // fill 5: 5 * 5 >= 7 * 3 -> set_table_resize to 32 slots
      constexpr int R = N > 4 ? 5 : N;   // N <= 4 never resizes (keeps the indices in range)
      uint64_t ks[5], kh[5];
      int kt[5];
#pragma unroll
      for (int i = 0; i < R; ++i) { ks[i] = slot[i]; kh[i] = h[i]; kt[i] = i; }
#pragma unroll
      for (int i = 0; i < 5; ++i)
#pragma unroll
        for (int q = 0; q < 4 - i; ++q)
          if (ks[q] > ks[q + 1]) {
            uint64_t tl = ks[q]; ks[q] = ks[q + 1]; ks[q + 1] = tl;
            tl = kh[q]; kh[q] = kh[q + 1]; kh[q + 1] = tl;
            const int ti = kt[q]; kt[q] = kt[q + 1]; kt[q + 1] = ti;
          }
      lo = ~0ULL; hi = ~0ULL;
      mask = 31;
#pragma unroll
      for (int i = 0; i < 5; ++i) pk_set(lo, hi, pk_probe(lo, hi, mask, kh[i]), kt[i]);
    }
  }
  uint32_t out = 0;
  int r = 0;
  for (uint64_t i = 0; i <= mask; ++i) {
    const int v = pk_get(lo, hi, i);
    if (v != 15) { out |= (uint32_t)v << (4 * r); ++r; }
  }
  return out;
}

}  // namespace pyset
