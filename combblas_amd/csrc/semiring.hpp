// semiring.hpp -- device semiring functors for the SpGEMM kernels.
//
// Each reference semiring is a static policy class (include/CombBLAS/Semirings.h); here each is a
// compile-time struct whose members the kernels call.  The accumulator ("Acc") is what lives in LDS
// hash/dense slots; for most semirings it is the value type itself, except:
//   * SELECT2ND keeps the *B position* of the first contributor (min over storage order, which is
//     exactly "first insert wins": Select2ndSRing::add returns arg2 = existing, Semirings.h:149-152,
//     called as add(new, existing) at mtSpGEMM.h:583) and the value is gathered at write-out;
//   * bool values are accumulated as int32 0/1 (LDS atomics are 32-bit).
// Every accumulate is an LDS atomic so lanes of a workgroup can hit the same slot concurrently.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <float.h>

namespace cbg {

enum : int { SR_PLUS_TIMES = 0, SR_MIN_PLUS = 1, SR_SELECT2ND = 2, SR_SELECT_MAX = 3,
             SR_SELECT_MAX_BOOL = 4, SR_BOOL_COPY1ST = 5, SR_BOOL_COPY2ND = 6 };

template <typename T> struct Lim;
template <> struct Lim<double>  { __device__ __host__ static constexpr double  max() { return DBL_MAX; }   __device__ __host__ static constexpr double  lowest() { return -DBL_MAX; } };
template <> struct Lim<float>   { __device__ __host__ static constexpr float   max() { return FLT_MAX; }   __device__ __host__ static constexpr float   lowest() { return -FLT_MAX; } };
template <> struct Lim<int64_t> { __device__ __host__ static constexpr int64_t max() { return INT64_MAX; } __device__ __host__ static constexpr int64_t lowest() { return INT64_MIN; } };
template <> struct Lim<int32_t> { __device__ __host__ static constexpr int32_t max() { return INT32_MAX; } __device__ __host__ static constexpr int32_t lowest() { return INT32_MIN; } };

// ---- LDS atomics on the accumulator types ------------------------------------------------------
__device__ inline void lds_add(double* p, double v) { atomicAdd(p, v); }        // ds_add_f64
__device__ inline void lds_add(float* p, float v) { atomicAdd(p, v); }          // ds_add_f32
__device__ inline void lds_add(int64_t* p, int64_t v) { atomicAdd((unsigned long long*)p, (unsigned long long)v); }
__device__ inline void lds_add(int32_t* p, int32_t v) { atomicAdd(p, v); }

__device__ inline void lds_min(int64_t* p, int64_t v) { atomicMin((long long*)p, (long long)v); }
__device__ inline void lds_min(int32_t* p, int32_t v) { atomicMin(p, v); }
__device__ inline void lds_max(int64_t* p, int64_t v) { atomicMax((long long*)p, (long long)v); }
__device__ inline void lds_max(int32_t* p, int32_t v) { atomicMax(p, v); }

template <typename F>
__device__ inline void lds_cas_loop(double* p, F f) {
  unsigned long long* q = (unsigned long long*)p;
  unsigned long long old = *q, assumed;
  do {
    assumed = old;
    double nv = f(__longlong_as_double((long long)assumed));
    if (__double_as_longlong(nv) == (long long)assumed) return;
    old = atomicCAS(q, assumed, (unsigned long long)__double_as_longlong(nv));
  } while (old != assumed);
}
template <typename F>
__device__ inline void lds_cas_loop(float* p, F f) {
  unsigned int* q = (unsigned int*)p;
  unsigned int old = *q, assumed;
  do {
    assumed = old;
    float nv = f(__uint_as_float(assumed));
    if (__float_as_uint(nv) == assumed) return;
    old = atomicCAS(q, assumed, __float_as_uint(nv));
  } while (old != assumed);
}
__device__ inline void lds_min(double* p, double v) { lds_cas_loop(p, [v](double o) { return v < o ? v : o; }); }
__device__ inline void lds_min(float* p, float v) { lds_cas_loop(p, [v](float o) { return v < o ? v : o; }); }
__device__ inline void lds_max(double* p, double v) { lds_cas_loop(p, [v](double o) { return v > o ? v : o; }); }
__device__ inline void lds_max(float* p, float v) { lds_cas_loop(p, [v](float o) { return v > o ? v : o; }); }

// ---- semiring policies ------------------------------------------------------------------------
// V  : value type of A, B and C (bool is carried as uint8 in memory)
// Acc: LDS accumulator type; identity(): value slots are initialised to it before accumulation.
// mul(a, b, pos): product of A value a and B value b, pos = global index of the B nonzero.
// acc(slot, x): slot = add(x, slot) atomically.  out(acc, Bval): final value written to C.
template <int SR, typename V> struct Semiring;

template <typename V> struct AccOf { using type = V; };
template <> struct AccOf<uint8_t> { using type = int32_t; };

template <typename V> struct Semiring<SR_PLUS_TIMES, V> {        // Semirings.h:212-233
  using Acc = typename AccOf<V>::type;
  static constexpr bool kAddIsError = false, kNeedsBPos = false;
  __device__ static Acc identity() { return Acc(0); }
  __device__ static Acc mul(V a, V b, int64_t, int64_t) {
    if constexpr (sizeof(V) == 1) return Acc((a != 0) & (b != 0));   // PlusTimes<bool,bool> = AND
    else return Acc(a) * Acc(b);
  }
  __device__ static void acc(Acc* s, Acc x) {
    if constexpr (sizeof(V) == 1) lds_max(s, x);                     // bool '+' = OR
    else lds_add(s, x);
  }
  __device__ static V out(Acc a, const V*, const V*) { return V(a); }
};

template <typename V> struct Semiring<SR_MIN_PLUS, V> {           // Semirings.h:235-255, inf_plus 40-47
  using Acc = typename AccOf<V>::type;
  static constexpr bool kAddIsError = false, kNeedsBPos = false;
  __device__ static Acc identity() { return Lim<Acc>::max(); }
  __device__ static Acc mul(V a, V b, int64_t, int64_t) {
    const Acc inf = Lim<Acc>::max();
    Acc x = Acc(a), y = Acc(b);
    if (x == inf || y == inf) return inf;
    return x + y;
  }
  __device__ static void acc(Acc* s, Acc x) { lds_min(s, x); }
  __device__ static V out(Acc a, const V*, const V*) { return V(a); }
};

template <typename V> struct Semiring<SR_SELECT_MAX, V> {         // Semirings.h:165-190
  using Acc = typename AccOf<V>::type;
  static constexpr bool kAddIsError = false, kNeedsBPos = false;
  __device__ static Acc identity() { return Lim<Acc>::lowest(); }
  __device__ static Acc mul(V a, V b, int64_t, int64_t) { return Acc(a) * Acc(b); }
  __device__ static void acc(Acc* s, Acc x) { lds_max(s, x); }
  __device__ static V out(Acc a, const V*, const V*) { return V(a); }
};

template <typename V> struct Semiring<SR_SELECT_MAX_BOOL, V> {    // SelectMaxSRing<bool,T2>, Semirings.h:191-210
  using Acc = typename AccOf<V>::type;
  static constexpr bool kAddIsError = false, kNeedsBPos = false;
  __device__ static Acc identity() { return Lim<Acc>::lowest(); }
  __device__ static Acc mul(V, V b, int64_t, int64_t) { return Acc(b); }
  __device__ static void acc(Acc* s, Acc x) { lds_max(s, x); }
  __device__ static V out(Acc a, const V*, const V*) { return V(a); }
};

template <typename V> struct Semiring<SR_SELECT2ND, V> {          // Semirings.h:143-163
  using Acc = int32_t;                                            // min B position (first insert)
  static constexpr bool kAddIsError = false, kNeedsBPos = true;
  __device__ static Acc identity() { return INT32_MAX; }
  __device__ static Acc mul(V, V, int64_t, int64_t pos) { return Acc(pos); }
  __device__ static void acc(Acc* s, Acc x) { lds_min(s, x); }
  __device__ static V out(Acc a, const V*, const V* bval) { return bval ? bval[a] : V(1); }
};

template <typename V> struct Semiring<SR_BOOL_COPY2ND, V> {       // Semirings.h:50-94 (A is bool)
  using Acc = int32_t;                                            // B position, single contributor
  static constexpr bool kAddIsError = true, kNeedsBPos = true;
  __device__ static Acc identity() { return INT32_MAX; }
  __device__ static Acc mul(V, V, int64_t, int64_t pos) { return Acc(pos); }
  __device__ static void acc(Acc* s, Acc x) { lds_min(s, x); }
  __device__ static V out(Acc a, const V*, const V* bval) { return bval ? bval[a] : V(1); }
};

template <typename V> struct Semiring<SR_BOOL_COPY1ST, V> {       // Semirings.h:96-141 (B is bool)
  using Acc = typename AccOf<V>::type;
  static constexpr bool kAddIsError = true, kNeedsBPos = false;
  __device__ static Acc identity() { return Lim<Acc>::lowest(); }
  __device__ static Acc mul(V a, V, int64_t, int64_t) { return Acc(a); }
  __device__ static void acc(Acc* s, Acc x) { lds_max(s, x); }
  __device__ static V out(Acc a, const V*, const V*) { return V(a); }
};

// ---- multiway merge as a product ------------------------------------------------------------
// MultiwayMerge(lists) (MultiwayMerge.h:411-526) is run as Acat * Sel, where Acat holds the k
// partial products side by side (column l*ncol + j) and Sel(:, j) selects rows {l*ncol + j}.  The
// "multiply" copies the partial's value; "add" is the wrapped semiring's add.  Duplicates are
// combined in list order (SerialMerge keeps SR::add(acc, next)); for SELECT2ND the first list that
// holds the entry wins: Acc packs (Sel position << 40 | Acat position) and the minimum is kept.
template <class SR> struct MergeOf;
template <int SRI, typename V> struct MergeOf<Semiring<SRI, V>> {
  using Base = Semiring<SRI, V>;
  using Acc = typename Base::Acc;
  static constexpr bool kAddIsError = Base::kAddIsError, kNeedsBPos = false;
  __device__ static Acc identity() { return Base::identity(); }
  __device__ static Acc mul(V a, V, int64_t, int64_t) { return Acc(a); }
  __device__ static void acc(Acc* s, Acc x) { Base::acc(s, x); }
  __device__ static V out(Acc a, const V*, const V*) { return V(a); }
};
template <typename V> struct MergeOf<Semiring<SR_SELECT2ND, V>> {
  using Acc = int64_t;
  static constexpr bool kAddIsError = false, kNeedsBPos = true;
  __device__ static Acc identity() { return INT64_MAX; }
  __device__ static Acc mul(V, V, int64_t q, int64_t bpos) { return (bpos << 40) | q; }
  __device__ static void acc(Acc* s, Acc x) { lds_min(s, x); }
  __device__ static V out(Acc a, const V* aval, const V*) {
    return aval ? aval[a & ((1LL << 40) - 1)] : V(1);
  }
};

}  // namespace cbg
