// grid.hip -- distributed SpGEMM over a layers x rows x cols grid of MI355X ranks (include/cbgpu.h).
//
// Reference drivers (include/CombBLAS/ParFriends.h): Mult_AnXBn_Synch 1004-1108, Mult_AnXBn_DoubleBuff
// 798-997, Mult_AnXBn_Overlap 1110-1235, Mult_AnXBn_SUMMA3D 2918-3208; 3DSpGEMM/SUMMALayer.h:24-97 and
// Reductions.h:36-155.  One formulation covers them all: the layer SUMMA (q stages of a row-group
// broadcast of the A piece and a column-group broadcast of the B piece, a local product, a merge)
// followed, with L > 1 layers, by the fiber all-to-all of layer column parts and a merge.
//
// MI355X-first choices:
//   * pieces, broadcast buffers and products stay in HBM (no SpTuples round trip per stage);
//   * with RCCL the broadcasts of stage k+1 are issued on a communication stream before stage k's
//     local product (double-buffered receive slots sized once per call), ordered by HIP events;
//   * the three arrays of a piece go out as one RCCL group (one launch, no packing copy);
//   * the fiber exchange is a grouped ncclSend/ncclRecv all-to-all-v of column counts, rows, values.
// A caller-provided transport (cbg_transport: MPI on the reference side, gloo in tests) runs the same
// schedule synchronously through host callbacks.
#include "spgemm_host.hpp"
#include <rccl/rccl.h>
#include <chrono>

namespace {

inline double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define NCCLCHK(x)                                                                                     \
  do {                                                                                                 \
    ncclResult_t r_ = (x);                                                                             \
    if (r_ != ncclSuccess) {                                                                           \
      fprintf(stderr, "cbgpu: %s failed: %s (%s:%d)\n", #x, ncclGetErrorString(r_), __FILE__, __LINE__); \
      return CBG_ECOMM;                                                                                \
    }                                                                                                  \
  } while (0)


// count[c] = cp[c+1] - cp[c]
__global__ void k_col_counts(int64_t n, const int64_t* __restrict__ cp, int64_t* __restrict__ cnt) {
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < n; c += (int64_t)gridDim.x * blockDim.x)
    cnt[c] = cp[c + 1] - cp[c];
}
// rebased column range: out[c] = cp[c0 + c] - cp[c0], c in [0, n]
__global__ void k_cp_rebase(int64_t n, const int64_t* __restrict__ cp, int64_t c0, int64_t* __restrict__ out) {
  const int64_t base = cp[c0];
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c <= n; c += (int64_t)gridDim.x * blockDim.x)
    out[c] = cp[c0 + c] - base;
}
// row split of a CSC at `cut` (rows are sorted per column): per column, entries below the cut
__global__ void k_row_cut(int64_t ncol, const int64_t* __restrict__ cp, const int32_t* __restrict__ ir, int32_t cut,
                          int64_t* __restrict__ lo_cnt) {
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < ncol; c += (int64_t)gridDim.x * blockDim.x)
    lo_cnt[c] = lower_bound_rows(ir, cp[c], cp[c + 1], cut) - cp[c];
}
// copy the two row halves; hi rows are rebased by -cut
template <typename T>
__global__ void __launch_bounds__(256) k_row_split(int64_t ncol, const int64_t* __restrict__ cp,
                                                   const int32_t* __restrict__ ir, const T* __restrict__ val,
                                                   int32_t cut, const int64_t* __restrict__ lcp,
                                                   const int64_t* __restrict__ hcp, int32_t* __restrict__ lir,
                                                   T* __restrict__ lval, int32_t* __restrict__ hir,
                                                   T* __restrict__ hval) {
  const int w = threadIdx.x / kWave, l = lane_id();
  for (int64_t c = blockIdx.x * 4 + w; c < ncol; c += (int64_t)gridDim.x * 4) {
    const int64_t s = cp[c], e = cp[c + 1], nl = lcp[c + 1] - lcp[c];
    for (int64_t q = s + l; q < e; q += kWave) {
      const int64_t k = q - s;
      if (k < nl) {
        lir[lcp[c] + k] = ir[q];
        if (val) lval[lcp[c] + k] = val[q];
      } else {
        hir[hcp[c] + k - nl] = ir[q] - cut;
        if (val) hval[hcp[c] + k - nl] = val[q];
      }
    }
  }
}

// hcp[c] = cp[c] - lcp[c]
__global__ void k_cp_sub(int64_t n, const int64_t* __restrict__ cp, const int64_t* __restrict__ lcp,
                         int64_t* __restrict__ hcp) {
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c <= n; c += (int64_t)gridDim.x * blockDim.x)
    hcp[c] = cp[c] - lcp[c];
}

// panel assembly: B pieces of one grid column stacked by rows (column c = piece 0's rows, then piece
// 1's rows + its row offset, ...), A pieces of one grid row side by side
__global__ void k_add_col_counts(int64_t n, const int64_t* __restrict__ cp, int64_t* __restrict__ cnt) {
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < n; c += (int64_t)gridDim.x * blockDim.x)
    cnt[c] += cp[c + 1] - cp[c];
}
template <typename T>
__global__ void __launch_bounds__(256) k_stack_rows(int64_t ncol, const int64_t* __restrict__ cp,
                                                    const int32_t* __restrict__ ir, const T* __restrict__ val,
                                                    int32_t roff, int64_t* __restrict__ cursor,
                                                    int32_t* __restrict__ oir, T* __restrict__ oval) {
  const int w = threadIdx.x / kWave, l = lane_id();
  for (int64_t c = blockIdx.x * 4 + w; c < ncol; c += (int64_t)gridDim.x * 4) {
    const int64_t s = cp[c], e = cp[c + 1], o = cursor[c];
    for (int64_t q = s + l; q < e; q += kWave) {
      oir[o + (q - s)] = ir[q] + roff;
      if (val) oval[o + (q - s)] = val[q];
    }
    if (l == 0) cursor[c] = o + (e - s);
  }
}

// lossless narrowing of f64 messages: values that survive a round trip through f32 bit for bit
__global__ void k_f32_inexact(int64_t n, const double* __restrict__ v, unsigned long long* __restrict__ bad) {
  unsigned long long c = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    c += __double_as_longlong((double)(float)v[i]) != __double_as_longlong(v[i]);
  c = (unsigned long long)wave_sum64((int64_t)c);
  if (lane_id() == 0 && c) atomicAdd(bad, c);
}
__global__ void k_f64_to_u16(int64_t n, const double* __restrict__ in, unsigned short* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (unsigned short)in[i];
}
__global__ void k_u16_to_f64(int64_t n, const unsigned short* __restrict__ in, double* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (double)in[i];
}
// Fiber rows as 16-bit gaps: within a column (rows ascending) entry i travels as d = row[i] - row[i-1] (the first
// as row - 0) when d <= kGapMax, else as the escape code and its absolute row in a side stream of int32 (offsets:
// a scan of the per-column escape counts, which ride in the high half of the column counts).  One wave per column.
constexpr unsigned kGapEsc = 0xFFFFu, kGapMax = 0xFFFEu;

// split received column headers (count | aux << 32) in place: aux -> aux[i], the count stays in hdr[i]
__global__ void k_split_hdr(int64_t n, int64_t* hdr, int64_t* __restrict__ aux) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t v = hdr[i];
    aux[i] = v >> 32;
    hdr[i] = v & 0xffffffffLL;
  }
}
// x[i] += base, i in [0, n)
__global__ void k_add_base(int64_t n, int64_t* __restrict__ x, int64_t base) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) x[i] += base;
}
// column headers of a message: count | aux << 32 (aux = escapes of the u16 gaps, or the column's varint row bytes)
__global__ void k_pack_hdr(int64_t n, const int64_t* __restrict__ cp, const int64_t* __restrict__ aux,
                           int64_t* __restrict__ hdr) {   // aux == nullptr: no aux
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    hdr[i] = (cp[i + 1] - cp[i]) | (aux ? aux[i] << 32 : 0);
}

// Varint fiber codes (LEB128: 7 bits per byte, high bit = another byte follows).  Rows travel as varint gaps
// (row - previous row in the column, the first as row - 0), integer values in [0, 2^32) as varint integers: a
// multiplicity-valued product's entry is ~2-3 bytes instead of 6 (u16 gap + f32).  Per column the sender counts
// the bytes of every candidate format in one pass (k_code_count) and the message takes the smallest.
__device__ __forceinline__ int vlen32(uint32_t x) {
  return 1 + (x >= (1u << 7)) + (x >= (1u << 14)) + (x >= (1u << 21)) + (x >= (1u << 28));
}
__device__ __forceinline__ bool as_u32(double x, uint32_t* u) {   // an integer in [0, 2^32), bit-exact round trip
  const bool in = x >= 0.0 && x <= 4294967295.0;                   // false for NaN
  *u = in ? (uint32_t)x : 0u;
  return in && __double_as_longlong((double)*u) == __double_as_longlong(x);
}

// The codec kernels take one column per wave and kCodeEpl consecutive entries per lane per step (a step = 256
// entries or 256 bytes): one wave scan per step instead of one per 64 entries, four loads in flight per lane.
constexpr int kCodeEpl = 4;
constexpr int kCodeStep = kCodeEpl * kWave;
// The codec kernels run in one-wave workgroups (4 KB of LDS at most): the fiber pipeline decodes a received chunk while
// the own columns multiply, and a one-wave workgroup fits beside the persistent heavy grid (152.7 KB of LDS and 16
// waves per CU) and in the CUs it leaves to the transfer.
constexpr int kCodecNT = kWave;
inline int codec_grid(int64_t ncol) { return (int)grid_for(ncol, 1, kMaxGrid * 8); }

// one wave per column: escapes of the u16 gaps, varint bytes of the row gaps, varint bytes of the values; over
// the message: bad[0] values that do not survive f32, bad[1] not u16, bad[2] not u32 integers
__global__ void __launch_bounds__(kCodecNT) k_code_count(int64_t ncol, const int64_t* __restrict__ cp,
                                                    const int32_t* __restrict__ ir, const double* __restrict__ val,
                                                    int64_t* __restrict__ esc, int64_t* __restrict__ rbytes,
                                                    int64_t* __restrict__ vbytes, unsigned long long* __restrict__ bad) {
  const int l = lane_id();
  int64_t b32 = 0, b16 = 0, bvar = 0;
  for (int64_t c = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kWave; c < ncol;
       c += ((int64_t)gridDim.x * blockDim.x) / kWave) {
    const int64_t s = cp[c], e = cp[c + 1];
    int64_t ne = 0, nr = 0, nv = 0;
    int32_t prev = 0;   // the row before the step (0 before the column's first entry)
    // the next step's rows and values are loaded while this step is counted (a long column is one wave's serial
    // walk: without the prefetch every step waits a full memory latency)
    int32_t rn[kCodeEpl];
    double xn[kCodeEpl];
    // unconditional loads from clamped addresses (a conditional load becomes a branch + an immediate wait: the
    // four loads of a step would go out one at a time)
    auto load = [&](int64_t b) {
#pragma unroll
      for (int k = 0; k < kCodeEpl; ++k) {
        const int64_t i = min(b + k, e - 1);
        rn[k] = ir[i];
        if (val) xn[k] = val[i];
      }
    };
    if (s < e) load(s + kCodeEpl * l);   // (an empty column has no address to clamp to)
    for (int64_t i0 = s; i0 < e; i0 += kCodeStep) {
      const int64_t base = i0 + kCodeEpl * l;
      int32_t r[kCodeEpl];
      double x[kCodeEpl];
#pragma unroll
      for (int k = 0; k < kCodeEpl; ++k) { r[k] = rn[k]; x[k] = val ? xn[k] : 0.0; }
      if (i0 + kCodeStep < e) load(base + kCodeStep);
      const int32_t up = (int32_t)dpp_prev_lane((uint32_t)r[kCodeEpl - 1]);
      const int32_t before = l == 0 ? prev : up;
#pragma unroll
      for (int k = 0; k < kCodeEpl; ++k) {
        if (base + k >= e) break;
        const int64_t d = (int64_t)r[k] - (k ? r[k - 1] : before);
        ne += d > (int64_t)kGapMax;
        nr += vlen32((uint32_t)d);
        if (val) {
          const double v = x[k];
          b32 += __double_as_longlong((double)(float)v) != __double_as_longlong(v);
          const bool in16 = v >= 0.0 && v <= 65535.0;
          b16 += !(in16 && __double_as_longlong((double)(unsigned short)v) == __double_as_longlong(v));
          uint32_t u;
          const bool ok = as_u32(v, &u);
          bvar += !ok;
          nv += ok ? vlen32(u) : 5;
        }
      }
      prev = (int32_t)last_lane((uint32_t)r[kCodeEpl - 1]);
    }
    ne = wave_sum64(ne);
    nr = wave_sum64(nr);
    nv = wave_sum64(nv);
    if (l == 0) {
      esc[c] = ne;
      rbytes[c] = nr;
      if (vbytes) vbytes[c] = nv;
    }
  }
  b32 = wave_sum64(b32);
  b16 = wave_sum64(b16);
  bvar = wave_sum64(bvar);
  if (l == 0 && b32) atomicAdd(bad, (unsigned long long)b32);
  if (l == 0 && b16) atomicAdd(bad + 1, (unsigned long long)b16);
  if (l == 0 && bvar) atomicAdd(bad + 2, (unsigned long long)bvar);
}

// MODE 0: row gaps of ir, MODE 1: values (u32 integers) of val -> varint bytes at off[c] of column c.  A step's codes
// are assembled in the wave's LDS slice (one wave scan places them), then copied out with coalesced byte stores.
template <int MODE>
__global__ void __launch_bounds__(kCodecNT) k_var_encode(int64_t ncol, const int64_t* __restrict__ cp,
                                                         const int32_t* __restrict__ ir, const double* __restrict__ val,
                                                         const int64_t* __restrict__ off, uint8_t* __restrict__ out) {
  __shared__ uint8_t stage[kCodecNT / kWave][kCodeStep * 5];
  const int l = lane_id();
  uint8_t* sb = stage[threadIdx.x / kWave];
  for (int64_t c = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kWave; c < ncol;
       c += ((int64_t)gridDim.x * blockDim.x) / kWave) {
    const int64_t s = cp[c], e = cp[c + 1];
    int64_t o = off[c];
    int32_t prev = 0;
    int32_t rn[kCodeEpl];   // the next step's rows (MODE 0) or values (MODE 1), loaded one step ahead
    double vn[kCodeEpl];
    auto load = [&](int64_t b) {   // clamped, unconditional (see k_code_count)
#pragma unroll
      for (int k = 0; k < kCodeEpl; ++k) {
        const int64_t i = min(b + k, e - 1);
        if (MODE == 0) rn[k] = ir[i];
        else vn[k] = val[i];
      }
    };
    if (s < e) load(s + kCodeEpl * l);   // (an empty column has no address to clamp to)
    for (int64_t i0 = s; i0 < e; i0 += kCodeStep) {
      const int64_t base = i0 + kCodeEpl * l;
      uint32_t x[kCodeEpl];
      int len[kCodeEpl];
      int tot = 0;
      int32_t r[kCodeEpl];
      double vv[kCodeEpl];
#pragma unroll
      for (int k = 0; k < kCodeEpl; ++k) {
        if (MODE == 0) r[k] = rn[k];
        else vv[k] = vn[k];
      }
      if (i0 + kCodeStep < e) load(base + kCodeStep);
      if (MODE == 0) {
        const int32_t up = (int32_t)dpp_prev_lane((uint32_t)r[kCodeEpl - 1]);
        const int32_t before = l == 0 ? prev : up;
#pragma unroll
        for (int k = 0; k < kCodeEpl; ++k) x[k] = (uint32_t)(r[k] - (k ? r[k - 1] : before));
        prev = (int32_t)last_lane((uint32_t)r[kCodeEpl - 1]);
      } else {
#pragma unroll
        for (int k = 0; k < kCodeEpl; ++k) {
          x[k] = 0;
          if (base + k < e) (void)as_u32(vv[k], &x[k]);
        }
      }
#pragma unroll
      for (int k = 0; k < kCodeEpl; ++k) {
        len[k] = base + k < e ? vlen32(x[k]) : 0;
        tot += len[k];
      }
      const int incl = dpp_incl_scan(tot);
      const int T = (int)last_lane((uint32_t)incl);
      int p = incl - tot;
#pragma unroll
      for (int k = 0; k < kCodeEpl; ++k)
        for (int b = 0; b < len[k]; ++b)
          sb[p++] = (uint8_t)(((x[k] >> (7 * b)) & 0x7Fu) | (b + 1 < len[k] ? 0x80u : 0u));
      wave_sync();
      for (int q = l; q < T; q += kWave) out[o + q] = sb[q];
      wave_sync();   // the slice is written again by the next step
      o += T;
    }
  }
}

// one wave per column: bytes [off[c], off[c+1]) -> entries [cp[c], cp[c+1]).  A step is 512 bytes, 8 per lane (the
// bytes in flight per wave are what bounds this kernel); a byte without the high bit ends an entry.  A code is at most 5
// bytes, so an entry ending in lane l's bytes starts in them or in the last 4 bytes of lane l-1's (lane 0: the previous
// step's lane 63, carried; at the column start the four bytes before it count as terminators).  MODE 0: the values are
// row gaps (scan + the column's running row -> int32 rows), MODE 1: u32 integers -> f64 values.  The next column's
// header is loaded while the current one is decoded.
constexpr int kDecEpl = 8;
constexpr int kDecStep = kDecEpl * kWave;
template <int MODE>
__global__ void __launch_bounds__(kCodecNT) k_var_decode(int64_t ncol, const int64_t* __restrict__ cp,
                                                         const int64_t* __restrict__ off, const uint8_t* __restrict__ in,
                                                         int32_t* __restrict__ ir, double* __restrict__ val) {
  // a step's decoded entries (<= 512) go through the wave's LDS slice and out with coalesced stores
  __shared__ uint64_t stage[kCodecNT / kWave][kDecStep];
  const int l = lane_id();
  uint64_t* sb = stage[threadIdx.x / kWave];
  const int64_t stride = ((int64_t)gridDim.x * blockDim.x) / kWave;
  int64_t c = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kWave;
  int64_t h_b = 0, h_e = 0, h_i = 0;   // the header of column c
  if (c < ncol) { h_b = off[c]; h_e = off[c + 1]; h_i = cp[c]; }
  for (; c < ncol; c += stride) {
    const int64_t b0 = h_b, be = h_e;
    int64_t idx = h_i;
    if (c + stride < ncol) { h_b = off[c + stride]; h_e = off[c + stride + 1]; h_i = cp[c + stride]; }
    int64_t run = 0;           // MODE 0: the last row decoded in this column
    uint32_t cw = 0, ctm = 0xFu;
    uint32_t bn[kDecEpl];   // the next step's bytes, loaded one step ahead
    auto load = [&](int64_t b) {   // clamped, unconditional (see k_code_count); masked where consumed
#pragma unroll
      for (int k = 0; k < kDecEpl; ++k) bn[k] = in[min(b + k, be - 1)];
    };
    if (b0 < be) load(b0 + kDecEpl * l);
    for (int64_t p0 = b0; p0 < be; p0 += kDecStep) {
      const int64_t pb = p0 + kDecEpl * l;
      uint64_t wd = 0;
      uint32_t tm = 0;
#pragma unroll
      for (int k = 0; k < kDecEpl; ++k) {
        const bool in_col = pb + k < be;
        const uint32_t b = in_col ? bn[k] : 0u;
        wd |= (uint64_t)b << (8 * k);
        tm |= (in_col && !(b & 0x80u) ? 1u : 0u) << k;
      }
      if (p0 + kDecStep < be) load(pb + kDecStep);
      const uint32_t hi = (uint32_t)(wd >> 32), thi = tm >> 4;
      uint32_t w1 = dpp_prev_lane(hi), t1 = dpp_prev_lane(thi);
      if (l == 0) { w1 = cw; t1 = ctm; }
      // window: positions 0..3 = lane l-1's last 4 bytes, 4..11 = this lane's 8 bytes
      const uint64_t W0 = (uint64_t)w1 | (wd << 32);
      const uint32_t W1 = hi;
      const uint32_t TM = t1 | (tm << 4);
      auto byte_at = [&](int p) -> uint32_t {
        return p < 8 ? (uint32_t)(W0 >> (8 * p)) & 0xFFu : (W1 >> (8 * (p - 8))) & 0xFFu;
      };
      uint32_t v[kDecEpl];
      int64_t g = 0;
#pragma unroll
      for (int k = 0; k < kDecEpl; ++k) {
        v[k] = 0;
        if ((tm >> k) & 1u) {
          const int q = 4 + k;
          const uint32_t below = TM & ((1u << q) - 1u);
          const int st = below ? 32 - __clz(below) : 0;   // one past the previous terminator
#pragma unroll
          for (int j = 0; j < 5; ++j)
            if (st + j <= q) v[k] |= (byte_at(st + j) & 0x7Fu) << (7 * j);
          g += v[k];
        }
      }
      const int cnt = __popc(tm);
      const int ci = dpp_incl_scan(cnt);
      const int T = (int)last_lane((uint32_t)ci);
      int at = ci - cnt;
      if (MODE == 0) {
        const int64_t gi = dpp_incl_scan64(g);
        int64_t row = run + (gi - g);
        uint32_t* s32 = (uint32_t*)sb;
#pragma unroll
        for (int k = 0; k < kDecEpl; ++k)
          if ((tm >> k) & 1u) {
            row += v[k];
            s32[at++] = (uint32_t)row;
          }
        run += last_lane64(gi);
        wave_sync();
        for (int q = l; q < T; q += kWave) ir[idx + q] = (int32_t)s32[q];
      } else {
        double* sd = (double*)sb;
#pragma unroll
        for (int k = 0; k < kDecEpl; ++k)
          if ((tm >> k) & 1u) sd[at++] = (double)v[k];
        wave_sync();
        for (int q = l; q < T; q += kWave) val[idx + q] = sd[q];
      }
      wave_sync();   // the slice is written again by the next step
      idx += T;
      cw = last_lane(hi);
      ctm = last_lane(thi);
    }
  }
}


// One pass instead of k_code_count + k_var_encode<0> + k_var_encode<1>: a wave per column counts every candidate form
// (escapes of the u16 gaps, the value checks) AND writes the varint codes of the row gaps and of the values into the
// column's worst-case slot (WR bytes per row gap: vlen of the largest row; 5 per value) at WR * cp[c] / 5 * cp[c], with
// the column's code bytes in rbytes[c] / vbytes[c].  k_compact_codes then packs the slots into the message (2.4 bytes
// per R-MAT entry read and written, against a second 12-byte read of the partial).  Value codes are written only when
// every value so far is a u32 integer (a message whose values do not code ships them in another form).
__global__ void __launch_bounds__(kCodecNT) k_code_encode(int64_t ncol, const int64_t* __restrict__ cp,
                                                          const int32_t* __restrict__ ir, const double* __restrict__ val,
                                                          int wr, uint8_t* __restrict__ rslot,
                                                          uint8_t* __restrict__ vslot, int64_t* __restrict__ esc,
                                                          int64_t* __restrict__ rbytes, int64_t* __restrict__ vbytes,
                                                          unsigned long long* __restrict__ bad) {
  __shared__ uint8_t stage[2][kCodeStep * 5];
  const int l = lane_id();
  int64_t b32 = 0, b16 = 0, bvar = 0;
  for (int64_t c = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kWave; c < ncol;
       c += ((int64_t)gridDim.x * blockDim.x) / kWave) {
    const int64_t s = cp[c], e = cp[c + 1];
    int64_t ne = 0, orow = 0, oval = 0;   // escapes; code bytes written so far (uniform)
    uint8_t* rdst = rslot + (int64_t)wr * s;
    uint8_t* vdst = vslot ? vslot + 5 * s : nullptr;
    int32_t prev = 0;
    int32_t rn[kCodeEpl];
    double xn[kCodeEpl];
    auto load = [&](int64_t b) {   // clamped, unconditional (see k_code_count)
#pragma unroll
      for (int k = 0; k < kCodeEpl; ++k) {
        const int64_t i = min(b + k, e - 1);
        rn[k] = ir[i];
        if (val) xn[k] = val[i];
      }
    };
    if (s < e) load(s + kCodeEpl * l);
    for (int64_t i0 = s; i0 < e; i0 += kCodeStep) {
      const int64_t base = i0 + kCodeEpl * l;
      int32_t r[kCodeEpl];
      double x[kCodeEpl];
#pragma unroll
      for (int k = 0; k < kCodeEpl; ++k) { r[k] = rn[k]; x[k] = val ? xn[k] : 0.0; }
      if (i0 + kCodeStep < e) load(base + kCodeStep);
      const int32_t up = (int32_t)dpp_prev_lane((uint32_t)r[kCodeEpl - 1]);
      const int32_t before = l == 0 ? prev : up;
      uint32_t g[kCodeEpl], u[kCodeEpl];
      int rl[kCodeEpl], vl[kCodeEpl];
      int rt = 0, vt = 0;
#pragma unroll
      for (int k = 0; k < kCodeEpl; ++k) {
        const bool in = base + k < e;
        const int64_t d = (int64_t)r[k] - (k ? r[k - 1] : before);
        g[k] = (uint32_t)d;
        ne += in && d > (int64_t)kGapMax;
        rl[k] = in ? vlen32(g[k]) : 0;
        rt += rl[k];
        u[k] = 0;
        vl[k] = 0;
        if (val && in) {
          const double v = x[k];
          b32 += __double_as_longlong((double)(float)v) != __double_as_longlong(v);
          const bool in16 = v >= 0.0 && v <= 65535.0;
          b16 += !(in16 && __double_as_longlong((double)(unsigned short)v) == __double_as_longlong(v));
          const bool ok = as_u32(v, &u[k]);
          bvar += !ok;
          vl[k] = ok ? vlen32(u[k]) : 5;
          vt += vl[k];
        }
      }
      prev = (int32_t)last_lane((uint32_t)r[kCodeEpl - 1]);
      // row codes: one wave scan places them in the row stage; value codes likewise in the value stage
      const int ri = dpp_incl_scan(rt);
      const int RT = (int)last_lane((uint32_t)ri);
      int p = ri - rt;
#pragma unroll
      for (int k = 0; k < kCodeEpl; ++k)
        for (int b = 0; b < rl[k]; ++b)
          stage[0][p++] = (uint8_t)(((g[k] >> (7 * b)) & 0x7Fu) | (b + 1 < rl[k] ? 0x80u : 0u));
      int VT = 0;
      if (vdst) {
        const int vi = dpp_incl_scan(vt);
        VT = (int)last_lane((uint32_t)vi);
        int q = vi - vt;
#pragma unroll
        for (int k = 0; k < kCodeEpl; ++k)
          for (int b = 0; b < vl[k]; ++b)
            stage[1][q++] = (uint8_t)(((u[k] >> (7 * b)) & 0x7Fu) | (b + 1 < vl[k] ? 0x80u : 0u));
      }
      wave_sync();
      for (int q = l; q < RT; q += kWave) rdst[orow + q] = stage[0][q];
      if (vdst)
        for (int q = l; q < VT; q += kWave) vdst[oval + q] = stage[1][q];
      wave_sync();   // the stages are written again by the next step
      orow += RT;
      oval += VT;
    }
    ne = wave_sum64(ne);
    if (l == 0) {
      esc[c] = ne;
      rbytes[c] = orow;
      if (vbytes) vbytes[c] = oval;
    }
  }
  b32 = wave_sum64(b32);
  b16 = wave_sum64(b16);
  bvar = wave_sum64(bvar);
  if (l == 0 && b32) atomicAdd(bad, (unsigned long long)b32);
  if (l == 0 && b16) atomicAdd(bad + 1, (unsigned long long)b16);
  if (l == 0 && bvar) atomicAdd(bad + 2, (unsigned long long)bvar);
}

// the columns' code slots (w bytes per entry, column c at w * cp[c]) packed into one stream at off[c] (a scan of
// the code bytes): a wave per column, consecutive lanes on consecutive bytes
__global__ void __launch_bounds__(kCodecNT) k_compact_codes(int64_t ncol, const int64_t* __restrict__ cp, int w,
                                                            const uint8_t* __restrict__ slot,
                                                            const int64_t* __restrict__ off, uint8_t* __restrict__ out) {
  const int l = lane_id();
  for (int64_t c = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kWave; c < ncol;
       c += ((int64_t)gridDim.x * blockDim.x) / kWave) {
    const uint8_t* src = slot + (int64_t)w * cp[c];
    const int64_t o = off[c], n = off[c + 1] - o;
    uint8_t* dst = out + o;
    int64_t q = l;
    for (; q + 3 * kWave < n; q += 4 * kWave) {   // four bytes in flight per lane
      const uint8_t b0 = src[q], b1 = src[q + kWave], b2 = src[q + 2 * kWave], b3 = src[q + 3 * kWave];
      dst[q] = b0; dst[q + kWave] = b1; dst[q + 2 * kWave] = b2; dst[q + 3 * kWave] = b3;
    }
    for (; q < n; q += kWave) dst[q] = src[q];
  }
}

__global__ void k_gap_encode(int64_t ncol, const int64_t* __restrict__ cp, const int32_t* __restrict__ ir,
                             const int64_t* __restrict__ eoff, unsigned short* __restrict__ gap,
                             int32_t* __restrict__ esc) {
  const int l = lane_id();
  for (int64_t c = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kWave; c < ncol;
       c += ((int64_t)gridDim.x * blockDim.x) / kWave) {
    const int64_t s = cp[c], e = cp[c + 1];
    int64_t eo = eoff[c];
    for (int64_t i0 = s; i0 < e; i0 += kWave) {
      const int64_t i = i0 + l;
      bool x = false;
      int32_t r = 0;
      if (i < e) {
        r = ir[i];
        const int64_t d = (int64_t)r - (i == s ? 0 : ir[i - 1]);
        x = d > (int64_t)kGapMax;
        gap[i] = x ? (unsigned short)kGapEsc : (unsigned short)d;
      }
      const uint64_t m = __ballot(x);
      if (x) esc[eo + __popcll(m & ((1ull << l) - 1))] = r;
      eo += __popcll(m);
    }
  }
}

// gap[i - gbase]: the gap stream of entries [gbase, ...) (one chunk of a message), cp absolute
__global__ void k_gap_decode(int64_t ncol, const int64_t* __restrict__ cp, const int64_t* __restrict__ eoff,
                             const unsigned short* __restrict__ gap, const int32_t* __restrict__ esc,
                             int32_t* __restrict__ ir, int64_t gbase) {
  const int l = lane_id();
  for (int64_t c = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kWave; c < ncol;
       c += ((int64_t)gridDim.x * blockDim.x) / kWave) {
    const int64_t s = cp[c], e = cp[c + 1];
    int64_t eo = eoff[c];
    int32_t carry = 0;   // the row before the chunk (0 before the column's first entry)
    for (int64_t i0 = s; i0 < e; i0 += kWave) {
      const int64_t i = i0 + l;
      const unsigned g = i < e ? gap[i - gbase] : 0u;
      const bool x = i < e && g == kGapEsc;
      const uint64_t m = __ballot(x);
      const int32_t a = x ? esc[eo + __popcll(m & ((1ull << l) - 1))] : 0;
      eo += __popcll(m);
      // inclusive scan of the gaps (escapes add 0), then each lane adds its last escape's row (or the carry)
      // minus the scan value at that escape
      int64_t sc = x ? 0 : (int64_t)g;
      sc = wave_incl_scan64(sc);
      const uint64_t upto = m & (l == 63 ? ~0ull : ((1ull << (l + 1)) - 1));
      const int le = upto ? 63 - __clzll(upto) : -1;   // last escape lane <= l
      const int32_t abs_le = __shfl(a, le < 0 ? 0 : le, kWave);
      const int64_t sc_le = __shfl(sc, le < 0 ? 0 : le, kWave);
      const int64_t row = le < 0 ? (int64_t)carry + sc : (int64_t)abs_le + (sc - sc_le);
      if (i < e) ir[i] = (int32_t)row;
      carry = (int32_t)__shfl(row, kWave - 1, kWave);
    }
  }
}

__global__ void k_f64_to_f32(int64_t n, const double* __restrict__ in, float* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (float)in[i];
}
__global__ void k_f32_to_f64(int64_t n, const float* __restrict__ in, double* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (double)in[i];
}

// a local product's own profile (cbg_profile of the call just made) into the rank's sums
void note_local(cbg_grid_stats* st, const cbg_ctx* ctx, const cbg_dcsc_view& vb) {
  if (!st) return;
  const cbg_profile& p = ctx->prof;
  st->heavy_ms += p.heavy_ms;
  st->heavy_multiplies += p.heavy_multiplies;
  st->heavy_nnz_b += p.heavy_nnz_b;
  st->heavy_nnz_c += p.heavy_nnz_c;
  st->local_nnz_out += p.nnz_out;
  st->local_nnz_b += vb.nnz;
  st->local_ncol_b += vb.ncol;
  ++st->local_products;
}

// device CSC piece (int64 colptr, int32 rows); storage owned by `own` unless borrowed
struct Piece {
  int64_t nrow = 0, ncol = 0, nnz = 0;
  const int64_t* cp = nullptr;
  const int32_t* ir = nullptr;
  const void* val = nullptr;
  std::shared_ptr<Owner> own;    // storage of cp/ir/val (or of cp only, see keep)
  std::shared_ptr<Owner> keep;   // shared storage the arrays point into (fiber receive buffers)
  int32_t k = 0, r = 0;          // stage (inner block) and half of the product: merge order
  bool reduced = false;          // already reduced over the fiber (fiber_pipeline)
};

}  // namespace

struct cbg_grid {
  cbg_ctx* ctx = nullptr;
  int world = 1, rank = 0, L = 1, q = 1, layer = 0, row = 0, col = 0;
  bool rccl = false;
  ncclComm_t comm[4] = {nullptr, nullptr, nullptr, nullptr};
  // a second fiber communicator for the fiber pipeline's per-chunk count exchanges: operations on one communicator
  // run in issue order, so on the data communicator chunk c+1's counts would wait behind chunk c's transfer
  ncclComm_t fiber_ctl = nullptr;
  cbg_transport cb{};
  hipStream_t cs = nullptr;          // communication stream
  hipStream_t ds = nullptr;          // fiber pipeline: decodes received chunks while the own columns multiply
  hipEvent_t ev_comm[2] = {}, ev_used[2] = {}, ev_t[4] = {};
  hipEvent_t ev_rx[8] = {};          // fiber pipeline: chunk c has arrived (recorded on cs after its transfer)
  std::vector<hipEvent_t> ev_stage;  // timing events of the schedules, created once and reused by every call
  hipError_t stage_event(size_t i, hipEvent_t* e) {
    while (ev_stage.size() <= i) {
      hipEvent_t x;
      hipError_t r = hipEventCreate(&x);
      if (r != hipSuccess) return r;
      ev_stage.push_back(x);
    }
    *e = ev_stage[i];
    return hipSuccess;
  }
  bool used_rec[2] = {false, false};
  DevBuf slotA[2], slotB[2], small, xsend, xrecv, xcnt;

  int gsize(int g) const { return g == CBG_GROUP_ROW || g == CBG_GROUP_COL ? q : g == CBG_GROUP_FIBER ? L : world; }
  int grank(int g) const { return g == CBG_GROUP_ROW ? col : g == CBG_GROUP_COL ? row : g == CBG_GROUP_FIBER ? layer : rank; }
};

namespace {

// ------------------------------------------------------------------------------------ transport
// n arrays broadcast from member `root` of group g (in place at the root); async on G->cs with RCCL
cbg_status t_bcast(cbg_grid* G, int g, int n, void* const* bufs, const int64_t* bytes, int root) {
  if (G->gsize(g) == 1) return CBG_OK;
  if (G->rccl) {
    NCCLCHK(ncclGroupStart());
    for (int i = 0; i < n; ++i)
      if (bytes[i] > 0) NCCLCHK(ncclBroadcast(bufs[i], bufs[i], (size_t)bytes[i], ncclInt8, root, G->comm[g], G->cs));
    NCCLCHK(ncclGroupEnd());
    return CBG_OK;
  }
  HIPCHK(hipStreamSynchronize(G->ctx->stream));
  HIPCHK(hipStreamSynchronize(G->cs));
  const bool me_root = G->grank(g) == root;
  for (int i = 0; i < n; ++i) {
    if (bytes[i] <= 0) continue;
    if (!G->cb.host_buffers) {
      if (G->cb.bcast(G->cb.user, g, bufs[i], bytes[i], root) != 0) return CBG_ECOMM;
      continue;
    }
    std::vector<char> h((size_t)bytes[i]);
    if (me_root) HIPCHK(hipMemcpy(h.data(), bufs[i], bytes[i], hipMemcpyDeviceToHost));
    if (G->cb.bcast(G->cb.user, g, h.data(), bytes[i], root) != 0) return CBG_ECOMM;
    if (!me_root) HIPCHK(hipMemcpy(bufs[i], h.data(), bytes[i], hipMemcpyHostToDevice));
  }
  return CBG_OK;
}

// all-to-all-v of device buffers over group g: segment m of `send` (sbytes[m]) goes to member m;
// segments land in member order in `recv`.  Synchronous on return.
cbg_status t_alltoallv(cbg_grid* G, int g, const void* send, const int64_t* sbytes, void* recv, const int64_t* rbytes,
                       ncclComm_t comm = nullptr) {
  const int P = G->gsize(g), me = G->grank(g);
  std::vector<int64_t> so(P + 1, 0), ro(P + 1, 0);
  for (int m = 0; m < P; ++m) { so[m + 1] = so[m] + sbytes[m]; ro[m + 1] = ro[m] + rbytes[m]; }
  hipStream_t st = G->ctx->stream;
  if (P == 1) {
    if (sbytes[0]) HIPCHK(hipMemcpyAsync(recv, send, sbytes[0], hipMemcpyDeviceToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
    return CBG_OK;
  }
  if (G->rccl) {
    if (sbytes[me]) HIPCHK(hipMemcpyAsync((char*)recv + ro[me], (const char*)send + so[me], sbytes[me],
                                          hipMemcpyDeviceToDevice, st));
    NCCLCHK(ncclGroupStart());
    for (int m = 0; m < P; ++m) {
      if (m == me) continue;
      if (sbytes[m]) NCCLCHK(ncclSend((const char*)send + so[m], (size_t)sbytes[m], ncclInt8, m, comm ? comm : G->comm[g], st));
      if (rbytes[m]) NCCLCHK(ncclRecv((char*)recv + ro[m], (size_t)rbytes[m], ncclInt8, m, comm ? comm : G->comm[g], st));
    }
    NCCLCHK(ncclGroupEnd());
    HIPCHK(hipStreamSynchronize(st));
    return CBG_OK;
  }
  HIPCHK(hipStreamSynchronize(st));
  if (!G->cb.host_buffers) return G->cb.alltoallv(G->cb.user, g, send, sbytes, recv, rbytes) == 0 ? CBG_OK : CBG_ECOMM;
  std::vector<char> hs((size_t)so[P] + 1), hr((size_t)ro[P] + 1);
  if (so[P]) HIPCHK(hipMemcpy(hs.data(), send, so[P], hipMemcpyDeviceToHost));
  if (G->cb.alltoallv(G->cb.user, g, hs.data(), sbytes, hr.data(), rbytes) != 0) return CBG_ECOMM;
  if (ro[P]) HIPCHK(hipMemcpy(recv, hr.data(), ro[P], hipMemcpyHostToDevice));
  return CBG_OK;
}

// all-gather of `bytes` host bytes per member (GetSetSizes); synchronous
cbg_status t_allgather(cbg_grid* G, int g, const void* mine, void* all, int64_t bytes) {
  const int P = G->gsize(g);
  if (P == 1) { memcpy(all, mine, bytes); return CBG_OK; }
  if (G->rccl) {
    HIPCHK(G->small.reserve(bytes * (P + 1)));
    char* d = G->small.as<char>();
    HIPCHK(hipMemcpyAsync(d, mine, bytes, hipMemcpyHostToDevice, G->cs));
    NCCLCHK(ncclAllGather(d, d + bytes, (size_t)bytes, ncclInt8, G->comm[g], G->cs));
    HIPCHK(hipMemcpyAsync(all, d + bytes, bytes * P, hipMemcpyDeviceToHost, G->cs));
    HIPCHK(hipStreamSynchronize(G->cs));
    return CBG_OK;
  }
  return G->cb.allgather(G->cb.user, g, mine, all, bytes) == 0 ? CBG_OK : CBG_ECOMM;
}

// every rank's flag -> true iff all are set (world all-gather of one int)
cbg_status all_ok(cbg_grid* G, bool mine, bool* out) {
  std::vector<int32_t> v(G->world);
  int32_t m = mine ? 1 : 0;
  CBGCHK(t_allgather(G, CBG_GROUP_WORLD, &m, v.data(), 4));
  *out = true;
  for (int32_t x : v) *out = *out && x;
  return CBG_OK;
}

// ------------------------------------------------------------------------------------ pieces
cbg_status make_piece(cbg_ctx* ctx, const cbg_dcsc_view* v, cbg_dtype dt, Piece* p) {
  const int pb = v->ptr_bytes ? v->ptr_bytes : v->idx_bytes;
  p->nrow = v->nrow; p->ncol = v->ncol; p->nnz = v->nnz;
  // a bool-typed operand of a non-bool product is a pattern (SelectMaxSRing<bool,T>, BoolCopy*)
  const bool pattern = !v->val || (v->val_type == CBG_BOOL && dt != CBG_BOOL);
  if (!pattern && v->val_type != dt) return CBG_EINVAL;
  if (v->on_device && !v->jc && pb == 8 && v->idx_bytes == 4) {   // zero copy
    p->cp = (const int64_t*)v->cp;
    p->ir = (const int32_t*)v->ir;
    p->val = pattern ? nullptr : v->val;
    return CBG_OK;
  }
  cbg_dcsc_view u = *v;
  if (pattern) u.val = nullptr;
  cbg_csc_result r;
  CBGCHK(cbg_upload(ctx, &u, &r));
  p->own.reset((Owner*)r._owner, [](Owner* o) { delete o; });
  p->cp = r.colptr; p->ir = r.row; p->val = pattern ? nullptr : r.val;
  return CBG_OK;
}

cbg_dcsc_view view_of(const Piece& p, cbg_dtype dt, bool has_val) {
  cbg_dcsc_view v{};
  v.nrow = p.nrow; v.ncol = p.ncol; v.nnz = p.nnz; v.nzc = p.ncol;
  v.cp = p.cp; v.jc = nullptr; v.ir = p.ir; v.idx_bytes = 4; v.ptr_bytes = 8;
  v.val = has_val ? p.val : nullptr; v.val_type = has_val ? dt : CBG_BOOL; v.on_device = 1;
  return v;
}

cbg_csc_result result_of(const Piece& p, cbg_dtype dt) {
  cbg_csc_result r{};
  r.nrow = p.nrow; r.ncol = p.ncol; r.nnz = p.nnz;
  r.colptr = (int64_t*)p.cp; r.row = (int32_t*)p.ir; r.val = (void*)p.val; r.val_type = dt;
  return r;
}

// Piece owning a library result (freed with the piece)
Piece piece_of_result(cbg_csc_result& r) {
  Piece p;
  p.nrow = r.nrow; p.ncol = r.ncol; p.nnz = r.nnz;
  p.cp = r.colptr; p.ir = r.row; p.val = r.val;
  p.own.reset((Owner*)r._owner, [](Owner* o) { delete o; });
  r._owner = nullptr;
  return p;
}

// columns [0, cut) and [cut, ncol) of a piece (Split by columns, SpDCCols.cpp:897)
cbg_status col_halves(cbg_ctx* ctx, const Piece& a, size_t vs, Piece* h) {
  const int64_t cut = a.ncol / 2;
  hipStream_t st = ctx->stream;
  int64_t e = 0;
  HIPCHK(hipMemcpyAsync(&e, a.cp + cut, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  h[0] = a; h[0].ncol = cut; h[0].nnz = e;   // prefix: same arrays, shorter colptr
  std::shared_ptr<Owner> o(new Owner(ctx->pool));
  HIPCHK(o->cp.reserve(8 * (a.ncol - cut + 1)));
  k_cp_rebase<<<(int)grid_for(a.ncol - cut + 1, 256, kMaxGrid), 256, 0, st>>>(a.ncol - cut, a.cp, cut, o->cp.as<int64_t>());
  HIPCHK(hipGetLastError());
  h[1] = a;
  h[1].ncol = a.ncol - cut; h[1].nnz = a.nnz - e;
  h[1].cp = o->cp.as<int64_t>(); h[1].ir = a.ir + e;
  h[1].val = a.val ? (const void*)((const char*)a.val + vs * e) : nullptr;
  h[1].own = o;
  return CBG_OK;
}

// rows [0, cut) and [cut, nrow) of a piece, the second rebased (Split after transpose, ParFriends.h:823-829)
template <typename T>
cbg_status row_halves(cbg_ctx* ctx, const Piece& b, Piece* h) {
  const int32_t cut = (int32_t)(b.nrow / 2);
  hipStream_t st = ctx->stream;
  std::shared_ptr<Owner> lo(new Owner(ctx->pool)), hi(new Owner(ctx->pool));
  PoolBuf cnt, tiles, scal;
  cnt.pool = tiles.pool = scal.pool = ctx->pool;
  const int64_t n = b.ncol;
  HIPCHK(cnt.reserve(8 * (2 * n + 2)));
  HIPCHK(lo->cp.reserve(8 * (n + 1)));
  HIPCHK(hi->cp.reserve(8 * (n + 1)));
  int64_t* lcnt = cnt.as<int64_t>();
  int64_t* hcnt = lcnt + n + 1;
  const int g = (int)grid_for(n, 256, kMaxGrid);
  int64_t tot[2] = {0, 0};
  if (n > 0) {
    k_row_cut<<<g, 256, 0, st>>>(n, b.cp, b.ir, cut, lcnt);
    k_col_counts<<<g, 256, 0, st>>>(n, b.cp, hcnt);
    const int64_t ntiles = (n + kScanTile - 1) / kScanTile;
    HIPCHK(tiles.reserve(8 * (ntiles + 1)));
    HIPCHK(scal.reserve(16));
    k_scan_tiles<<<(int)ntiles, 256, 0, st>>>(n, lcnt, tiles.as<int64_t>());
    k_scan_sums<<<1, 1024, 0, st>>>(ntiles, tiles.as<int64_t>(), scal.as<int64_t>());
    k_scan_apply<<<(int)ntiles, 256, 0, st>>>(n, lcnt, tiles.as<int64_t>(), lo->cp.as<int64_t>());
    // hi counts = total - lo
    HIPCHK(hipMemcpyAsync(&tot[0], scal.p, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  } else {
    HIPCHK(hipMemsetAsync(lo->cp.p, 0, 8, st));
  }
  tot[1] = b.nnz - tot[0];
  k_cp_sub<<<(int)grid_for(n + 1, 256, kMaxGrid), 256, 0, st>>>(n, b.cp, lo->cp.as<int64_t>(), hi->cp.as<int64_t>());
  HIPCHK(lo->ir.reserve(4 * (tot[0] + 1)));
  HIPCHK(hi->ir.reserve(4 * (tot[1] + 1)));
  HIPCHK(lo->val.reserve(sizeof(T) * (tot[0] + 1)));
  HIPCHK(hi->val.reserve(sizeof(T) * (tot[1] + 1)));
  if (n > 0 && b.nnz > 0)
    k_row_split<T><<<(int)grid_for(n, 4, kMaxGrid * 2), 256, 0, st>>>(
        n, b.cp, b.ir, (const T*)b.val, cut, lo->cp.as<int64_t>(), hi->cp.as<int64_t>(), lo->ir.as<int32_t>(),
        lo->val.as<T>(), hi->ir.as<int32_t>(), hi->val.as<T>());
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(st));   // cnt/tiles/scal go back to the pool on return
  h[0].nrow = cut; h[0].ncol = n; h[0].nnz = tot[0];
  h[0].cp = lo->cp.as<int64_t>(); h[0].ir = lo->ir.as<int32_t>(); h[0].val = b.val ? lo->val.p : nullptr; h[0].own = lo;
  h[1].nrow = b.nrow - cut; h[1].ncol = n; h[1].nnz = tot[1];
  h[1].cp = hi->cp.as<int64_t>(); h[1].ir = hi->ir.as<int32_t>(); h[1].val = b.val ? hi->val.p : nullptr; h[1].own = hi;
  return CBG_OK;
}

cbg_status row_halves_dt(cbg_ctx* ctx, cbg_dtype dt, const Piece& b, Piece* h) {
  switch (dt_size(dt)) {
    case 1: return row_halves<uint8_t>(ctx, b, h);
    case 4: return row_halves<uint32_t>(ctx, b, h);
    default: return row_halves<uint64_t>(ctx, b, h);
  }
}

// move a pool block between owners (PoolBuf returns its block to the pool on destruction)
void take(PoolBuf& dst, PoolBuf& src) {
  std::swap(dst.p, src.p);
  std::swap(dst.n, src.n);
  std::swap(dst.pool, src.pool);
}

struct Sizes {   // GetSetSizes record of one piece
  int64_t nrow, ncol, nnz, has_val;
};

// merge device results (cbg_merge) into one library result; parts are borrowed
cbg_status merge_parts(cbg_ctx* ctx, const std::vector<cbg_csc_result>& parts, cbg_semiring sr, cbg_dtype dt,
                       cbg_csc_result* out) {
  return cbg_merge(ctx, parts.data(), (int32_t)parts.size(), sr, dt, CBG_SORTED_COLS, out);
}

// ------------------------------------------------------------------------------------ layer SUMMA
// Internal flag: the layer's product as ONE local multiply of its panels (below).
constexpr uint32_t kPanels = 1u << 30;

// A panel: the q A pieces of the grid row side by side (inner blocks 0..q-1)
cbg_status panel_cols(cbg_ctx* ctx, const std::vector<Piece>& a, size_t vs, bool has_val, Piece* out) {
  hipStream_t st = ctx->stream;
  int64_t ncol = 0, nnz = 0;
  for (const Piece& p : a) { ncol += p.ncol; nnz += p.nnz; }
  std::shared_ptr<Owner> o(new Owner(ctx->pool));
  HIPCHK(o->cp.reserve(8 * (ncol + 1)));
  HIPCHK(o->ir.reserve(4 * (nnz + 1)));
  HIPCHK(o->val.reserve(vs * (nnz + 1) + 8));
  int64_t c0 = 0, e0 = 0;
  for (const Piece& p : a) {
    if (p.ncol) k_merge_cat_cp<<<(int)grid_for(p.ncol, 256, kMaxGrid), 256, 0, st>>>(p.ncol, p.cp, e0, o->cp.as<int64_t>() + c0);
    if (p.nnz) {
      HIPCHK(hipMemcpyAsync(o->ir.as<int32_t>() + e0, p.ir, 4 * p.nnz, hipMemcpyDeviceToDevice, st));
      if (has_val) HIPCHK(hipMemcpyAsync(o->val.as<char>() + vs * e0, p.val, vs * p.nnz, hipMemcpyDeviceToDevice, st));
    }
    c0 += p.ncol;
    e0 += p.nnz;
  }
  HIPCHK(hipMemcpyAsync(o->cp.as<int64_t>() + ncol, &nnz, 8, hipMemcpyHostToDevice, st));
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(st));   // `nnz` above is a host temporary
  out->nrow = a[0].nrow; out->ncol = ncol; out->nnz = nnz;
  out->cp = o->cp.as<int64_t>(); out->ir = o->ir.as<int32_t>(); out->val = has_val ? o->val.p : nullptr;
  out->own = o;
  return CBG_OK;
}

// B panel: the q B pieces of the grid column stacked by rows (inner blocks 0..q-1)
template <typename T>
cbg_status panel_rows(cbg_ctx* ctx, const std::vector<Piece>& b, bool has_val, Piece* out) {
  hipStream_t st = ctx->stream;
  const int64_t ncol = b[0].ncol;
  int64_t nrow = 0, nnz = 0;
  for (const Piece& p : b) { nrow += p.nrow; nnz += p.nnz; }
  std::shared_ptr<Owner> o(new Owner(ctx->pool));
  HIPCHK(o->cp.reserve(8 * (ncol + 1)));
  HIPCHK(o->ir.reserve(4 * (nnz + 1)));
  HIPCHK(o->val.reserve(sizeof(T) * (nnz + 1)));
  PoolBuf cnt, tiles, scal;
  cnt.pool = tiles.pool = scal.pool = ctx->pool;
  HIPCHK(cnt.reserve(8 * (ncol + 1)));
  HIPCHK(hipMemsetAsync(cnt.p, 0, 8 * (ncol + 1), st));
  const int g = (int)grid_for(ncol, 256, kMaxGrid);
  for (const Piece& p : b)
    if (ncol) k_add_col_counts<<<g, 256, 0, st>>>(ncol, p.cp, cnt.as<int64_t>());
  const int64_t ntiles = (ncol + kScanTile - 1) / kScanTile;
  HIPCHK(tiles.reserve(8 * (ntiles + 1)));
  HIPCHK(scal.reserve(16));
  if (ncol > 0) {
    k_scan_tiles<<<(int)ntiles, 256, 0, st>>>(ncol, cnt.as<int64_t>(), tiles.as<int64_t>());
    k_scan_sums<<<1, 1024, 0, st>>>(ntiles, tiles.as<int64_t>(), scal.as<int64_t>());
    k_scan_apply<<<(int)ntiles, 256, 0, st>>>(ncol, cnt.as<int64_t>(), tiles.as<int64_t>(), o->cp.as<int64_t>());
    HIPCHK(hipMemcpyAsync(cnt.p, o->cp.p, 8 * ncol, hipMemcpyDeviceToDevice, st));   // cursors
  } else {
    HIPCHK(hipMemsetAsync(o->cp.p, 0, 8, st));
  }
  int32_t roff = 0;
  for (const Piece& p : b) {   // in inner-block order: the stacked rows stay sorted per column
    if (ncol && p.nnz)
      k_stack_rows<T><<<(int)grid_for(ncol, 4, kMaxGrid * 2), 256, 0, st>>>(
          ncol, p.cp, p.ir, has_val ? (const T*)p.val : nullptr, roff, cnt.as<int64_t>(), o->ir.as<int32_t>(),
          o->val.as<T>());
    roff += (int32_t)p.nrow;
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(st));   // cnt/tiles/scal go back to the pool on return
  out->nrow = nrow; out->ncol = ncol; out->nnz = nnz;
  out->cp = o->cp.as<int64_t>(); out->ir = o->ir.as<int32_t>(); out->val = has_val ? o->val.p : nullptr;
  out->own = o;
  return CBG_OK;
}

cbg_status panel_rows_dt(cbg_ctx* ctx, cbg_dtype dt, const std::vector<Piece>& b, bool has_val, Piece* out) {
  switch (dt_size(dt)) {
    case 1: return panel_rows<uint8_t>(ctx, b, has_val, out);
    case 4: return panel_rows<uint32_t>(ctx, b, has_val, out);
    default: return panel_rows<uint64_t>(ctx, b, has_val, out);
  }
}

cbg_status fiber_pipeline(cbg_grid* G, const cbg_dcsc_view& va, const cbg_dcsc_view& vb, cbg_semiring sr,
                          cbg_dtype dt, Piece* out, cbg_grid_stats* st);
cbg_status fiber_gather(cbg_grid* G, const cbg_dcsc_view& va, const cbg_dcsc_view& vb, cbg_semiring sr,
                        cbg_dtype dt, Piece* out, cbg_grid_stats* st);
cbg_status fiber_gather_ok(cbg_grid* G, const cbg_dcsc_view& va, const cbg_dcsc_view& vb, size_t vs, bool* out);
// The two-layer plain product's fiber step: the operand gather when every rank finds it cheaper (fiber_gather_ok),
// else the reduction pipeline.  CBG_FIBER_GATHER=0 always takes the reduction.
cbg_status fiber_step(cbg_grid* G, const cbg_dcsc_view& va, const cbg_dcsc_view& vb, cbg_semiring sr, cbg_dtype dt,
                      Piece* out, cbg_grid_stats* st) {
  static const bool gather_env = [] { const char* e = std::getenv("CBG_FIBER_GATHER"); return !(e && e[0] == '0'); }();
  bool gather = false;
  if (gather_env) CBGCHK(fiber_gather_ok(G, va, vb, dt_size(dt), &gather));
  return gather ? fiber_gather(G, va, vb, sr, dt, out, st) : fiber_pipeline(G, va, vb, sr, dt, out, st);
}
// Internal flag: L = 2, plain product -- the layer product runs in two column halves with the fiber exchange
// of the other layer's half overlapping the own half (fiber_pipeline); parts then holds the reduced piece.
constexpr uint32_t kFiberPipe = 1u << 29;
// CUs the own-half product leaves to RCCL while the fiber transfer is in flight (CBG_FIBER_RESERVE_CU overrides)
constexpr int kFiberReserveCu = 16;   // tools/coresidency_probe.py, profiles/r04a_coresidency_probe.jsonl

// est != nullptr: count only (EstPerProcessNnzSUMMA) -- every stage runs the symbolic pass alone and est[0] / est[1]
// accumulate its multiplies and nnz; no product is formed (staged schedule, parts stays empty)
cbg_status summa_layer_impl(cbg_grid* G, const cbg_dcsc_view* Av, const cbg_dcsc_view* Bv, cbg_semiring sr,
                            cbg_dtype dt, uint32_t flags, std::vector<Piece>* parts, cbg_grid_stats* st,
                            int64_t* est = nullptr) {
  cbg_ctx* ctx = G->ctx;
  const size_t vs = dt_size(dt);
  Piece A0, B0;
  CBGCHK(make_piece(ctx, Av, dt, &A0));
  CBGCHK(make_piece(ctx, Bv, dt, &B0));
  const bool aval = A0.val != nullptr, bval = B0.val != nullptr;
  // rounds: one, or two halves of the inner dimension (DoubleBuff)
  const int R = (flags & CBG_HALVES) ? 2 : 1;
  std::vector<Piece> Ah(R), Bh(R);
  if (R == 1) {
    Ah[0] = A0; Bh[0] = B0;
  } else {
    Piece h[2];
    CBGCHK(col_halves(ctx, A0, vs, h));
    Ah[0] = h[0]; Ah[1] = h[1];
    Piece g2[2];
    CBGCHK(row_halves_dt(ctx, dt, B0, g2));
    Bh[0] = g2[0]; Bh[1] = g2[1];
  }
  const int q = G->q;
  // GetSetSizes: every member's piece sizes (per round) in the row group (A) and column group (B)
  std::vector<Sizes> myA(R), myB(R), allA((size_t)R * q), allB((size_t)R * q);
  for (int r = 0; r < R; ++r) {
    // has_val: 1 values, 0 pattern, -1 empty (an empty piece's value pointer says nothing)
    myA[r] = Sizes{Ah[r].nrow, Ah[r].ncol, Ah[r].nnz, Ah[r].nnz ? (aval ? 1 : 0) : -1};
    myB[r] = Sizes{Bh[r].nrow, Bh[r].ncol, Bh[r].nnz, Bh[r].nnz ? (bval ? 1 : 0) : -1};
  }
  CBGCHK(t_allgather(G, CBG_GROUP_ROW, myA.data(), allA.data(), (int64_t)sizeof(Sizes) * R));
  CBGCHK(t_allgather(G, CBG_GROUP_COL, myB.data(), allB.data(), (int64_t)sizeof(Sizes) * R));
  auto SA = [&](int r, int k) -> const Sizes& { return allA[(size_t)k * R + r]; };
  auto SB = [&](int r, int k) -> const Sizes& { return allB[(size_t)k * R + r]; };
  // CheckSpGEMMCompliance (ParFriends.h:160-181) for every stage, agreed over the world
  bool ok = true;
  int64_t ha = -1, hb = -1;   // value/pattern status of the non-empty pieces: must agree
  for (int r = 0; r < R; ++r)
    for (int k = 0; k < q; ++k) {
      ok = ok && SA(r, k).ncol == SB(r, k).nrow && SA(r, k).nrow == SA(0, 0).nrow && SB(r, k).ncol == SB(0, 0).ncol;
      const int64_t a = SA(r, k).has_val, b = SB(r, k).has_val;
      if (a >= 0) { ok = ok && (ha < 0 || ha == a); ha = a; }
      if (b >= 0) { ok = ok && (hb < 0 || hb == b); hb = b; }
    }
  bool all = true;
  CBGCHK(all_ok(G, ok, &all));
  if (!all) return CBG_EDIM;
  // receive slots sized for the largest stage
  auto bytes_of = [&](const Sizes& s) -> int64_t { return 8 * (s.ncol + 1) + ((4 * s.nnz + 15) & ~15LL) + (int64_t)vs * s.nnz + 16; };
  int64_t needA = 16, needB = 16;
  for (int r = 0; r < R; ++r)
    for (int k = 0; k < q; ++k) {
      if (k != G->col) needA = std::max(needA, bytes_of(SA(r, k)));
      if (k != G->row) needB = std::max(needB, bytes_of(SB(r, k)));
    }
  bool panels = (flags & kPanels) && R == 1 && q > 1 && !est;
  if (panels) {
    // the panels hold the q received pieces of A and of B plus their concatenated copies; fall back to the
    // staged schedule (two receive slots) when that does not fit in the free HBM with room for the product
    int64_t need = 0;
    for (int k = 0; k < q; ++k) need += 2 * (bytes_of(SA(0, k)) + bytes_of(SB(0, k)));
    size_t freeb = 0, totalb = 0;
    if (hipMemGetInfo(&freeb, &totalb) == hipSuccess && (double)need > 0.5 * (double)freeb) panels = false;
    bool all_panels = true;   // every rank must take the same schedule (the collectives differ)
    CBGCHK(all_ok(G, panels, &all_panels));
    panels = all_panels;
  }
  if (panels) {
    // Panels: HBM holds the whole grid row of A and grid column of B (1/q of each operand), so the
    // layer's product is ONE local multiply of A(i, :) and B(:, j) -- the same bytes as the q stage
    // broadcasts, no stage products and no stage merge.  The inner blocks are concatenated in stage order,
    // so every duplicate combines in the order the staged merge would (Select2nd: first stage wins).
    std::vector<PoolBuf> bufA(q), bufB(q);
    StreamFence fence(G->cs, ctx->stream);   // broadcasts into bufA/bufB end before the buffers return to the pool
    std::vector<Piece> pa(q), pb(q);
    for (int k = 0; k < q; ++k) {
      Piece a, b;
      if (k == G->col) {
        a = A0;
      } else {
        const Sizes& z = SA(0, k);
        bufA[k].pool = ctx->pool;
        HIPCHK(bufA[k].reserve(bytes_of(z)));
        char* base = bufA[k].as<char>();
        a.nrow = z.nrow; a.ncol = z.ncol; a.nnz = z.nnz;
        a.cp = (const int64_t*)base;
        a.ir = (const int32_t*)(base + 8 * (z.ncol + 1));
        a.val = z.has_val > 0 ? (const void*)(base + 8 * (z.ncol + 1) + ((4 * z.nnz + 15) & ~15LL)) : nullptr;
      }
      if (k == G->row) {
        b = B0;
      } else {
        const Sizes& z = SB(0, k);
        bufB[k].pool = ctx->pool;
        HIPCHK(bufB[k].reserve(bytes_of(z)));
        char* base = bufB[k].as<char>();
        b.nrow = z.nrow; b.ncol = z.ncol; b.nnz = z.nnz;
        b.cp = (const int64_t*)base;
        b.ir = (const int32_t*)(base + 8 * (z.ncol + 1));
        b.val = z.has_val > 0 ? (const void*)(base + 8 * (z.ncol + 1) + ((4 * z.nnz + 15) & ~15LL)) : nullptr;
      }
      pa[k] = a;
      pb[k] = b;
    }
    hipEvent_t e0, e1, ready;
    HIPCHK(G->stage_event(0, &e0));
    HIPCHK(G->stage_event(1, &e1));
    HIPCHK(G->stage_event(2, &ready));
    HIPCHK(hipEventRecord(ready, ctx->stream));   // the own pieces are complete before they are sent
    HIPCHK(hipStreamWaitEvent(G->cs, ready, 0));
    HIPCHK(hipEventRecord(e0, G->cs));
    for (int k = 0; k < q; ++k) {
      void* ab[3] = {(void*)pa[k].cp, (void*)pa[k].ir, (void*)pa[k].val};
      int64_t an[3] = {8 * (pa[k].ncol + 1), 4 * pa[k].nnz, pa[k].val ? (int64_t)vs * pa[k].nnz : 0};
      void* bb[3] = {(void*)pb[k].cp, (void*)pb[k].ir, (void*)pb[k].val};
      int64_t bn[3] = {8 * (pb[k].ncol + 1), 4 * pb[k].nnz, pb[k].val ? (int64_t)vs * pb[k].nnz : 0};
      CBGCHK(t_bcast(G, CBG_GROUP_ROW, 3, ab, an, k));
      CBGCHK(t_bcast(G, CBG_GROUP_COL, 3, bb, bn, k));
      if (st) st->bcast_bytes += (k == G->col ? 0 : an[0] + an[1] + an[2]) + (k == G->row ? 0 : bn[0] + bn[1] + bn[2]);
    }
    HIPCHK(hipEventRecord(e1, G->cs));
    HIPCHK(hipStreamWaitEvent(ctx->stream, e1, 0));
    const double t0 = now_ms();
    Piece AP, BP;
    CBGCHK(panel_cols(ctx, pa, vs, ha > 0, &AP));
    CBGCHK(panel_rows_dt(ctx, dt, pb, hb > 0, &BP));
    pa.clear();
    pb.clear();
    cbg_dcsc_view va = view_of(AP, dt, AP.val != nullptr);
    cbg_dcsc_view vb = view_of(BP, dt, BP.val != nullptr);
    if (flags & kFiberPipe) {   // product + fiber reduction, overlapped
      Piece P;
      CBGCHK(fiber_step(G, va, vb, sr, dt, &P, st));
      if (st) st->stages += q;
      parts->push_back(P);
    } else {
      cbg_csc_result C;
      int64_t m = 0;
      CBGCHK(cbg_spgemm_local(ctx, &va, &vb, sr, dt, CBG_SORTED_COLS, &C, &m));
      note_local(st, ctx, vb);
      if (st) { st->multiplies += m; st->local_ms += now_ms() - t0; st->stages += q; }
      Piece P = piece_of_result(C);
      parts->push_back(P);
    }
    HIPCHK(hipStreamSynchronize(G->cs));
    HIPCHK(hipStreamSynchronize(ctx->stream));   // panels and receive buffers go back to the pool on return
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (st) st->bcast_ms += ms;
    return CBG_OK;
  }
  if (q > 1)
    for (int s = 0; s < 2; ++s) { HIPCHK(G->slotA[s].reserve(needA)); HIPCHK(G->slotB[s].reserve(needB)); }
  const int S = R * q;
  std::vector<Piece> recvA(S), recvB(S);
  std::vector<std::pair<hipEvent_t, hipEvent_t>> bev;
  // stage t = r*q + k: receive (or own) pieces, broadcasts issued on the comm stream
  auto issue = [&](int t) -> cbg_status {
    const int r = t / q, k = t % q, slot = t & 1;
    Piece a, b;
    if (k == G->col) {
      a = Ah[r];
    } else {
      const Sizes& s = SA(r, k);
      char* base = G->slotA[slot].as<char>();
      a.nrow = s.nrow; a.ncol = s.ncol; a.nnz = s.nnz;
      a.cp = (const int64_t*)base;
      a.ir = (const int32_t*)(base + 8 * (s.ncol + 1));
      a.val = s.has_val > 0 ? (const void*)(base + 8 * (s.ncol + 1) + ((4 * s.nnz + 15) & ~15LL)) : nullptr;
    }
    if (k == G->row) {
      b = Bh[r];
    } else {
      const Sizes& s = SB(r, k);
      char* base = G->slotB[slot].as<char>();
      b.nrow = s.nrow; b.ncol = s.ncol; b.nnz = s.nnz;
      b.cp = (const int64_t*)base;
      b.ir = (const int32_t*)(base + 8 * (s.ncol + 1));
      b.val = s.has_val > 0 ? (const void*)(base + 8 * (s.ncol + 1) + ((4 * s.nnz + 15) & ~15LL)) : nullptr;
    }
    if (q > 1) {
      hipEvent_t e0, e1;
      HIPCHK(G->stage_event(2 * (size_t)t, &e0));
      HIPCHK(G->stage_event(2 * (size_t)t + 1, &e1));
      if (G->rccl && G->used_rec[slot]) HIPCHK(hipStreamWaitEvent(G->cs, G->ev_used[slot], 0));
      HIPCHK(hipEventRecord(e0, G->cs));
      void* ab[3] = {(void*)a.cp, (void*)a.ir, (void*)a.val};
      int64_t an[3] = {8 * (a.ncol + 1), 4 * a.nnz, a.val ? (int64_t)vs * a.nnz : 0};
      void* bb[3] = {(void*)b.cp, (void*)b.ir, (void*)b.val};
      int64_t bn[3] = {8 * (b.ncol + 1), 4 * b.nnz, b.val ? (int64_t)vs * b.nnz : 0};
      CBGCHK(t_bcast(G, CBG_GROUP_ROW, 3, ab, an, k));
      CBGCHK(t_bcast(G, CBG_GROUP_COL, 3, bb, bn, k));
      HIPCHK(hipEventRecord(e1, G->cs));
      HIPCHK(hipEventRecord(G->ev_comm[slot], G->cs));
      bev.emplace_back(e0, e1);
      if (st) st->bcast_bytes += (k == G->col ? 0 : an[0] + an[1] + an[2]) + (k == G->row ? 0 : bn[0] + bn[1] + bn[2]);
    }
    recvA[t] = a;
    recvB[t] = b;
    return CBG_OK;
  };
  hipStream_t cst = ctx->stream;
  if ((flags & kFiberPipe) && S == 1 && !est) {   // one stage (q = 1): the own pieces, product + fiber overlapped
    cbg_dcsc_view va = view_of(Ah[0], dt, Ah[0].val != nullptr);
    cbg_dcsc_view vb = view_of(Bh[0], dt, Bh[0].val != nullptr);
    Piece P;
    CBGCHK(fiber_step(G, va, vb, sr, dt, &P, st));
    if (st) ++st->stages;
    parts->push_back(P);
    return CBG_OK;
  }
  const bool async = G->rccl && q > 1;
  if (async) CBGCHK(issue(0));
  std::vector<Piece> acc;   // running merge (Overlap)
  for (int t = 0; t < S; ++t) {
    if (async) {
      if (t + 1 < S) CBGCHK(issue(t + 1));
      HIPCHK(hipStreamWaitEvent(cst, G->ev_comm[t & 1], 0));
    } else {
      CBGCHK(issue(t));
    }
    const double t0 = now_ms();
    cbg_dcsc_view va = view_of(recvA[t], dt, recvA[t].val != nullptr);
    cbg_dcsc_view vb = view_of(recvB[t], dt, recvB[t].val != nullptr);
    if (est) {   // symbolic pass only (estimateFLOP + estimateNNZ_Hash of the stage, ParFriends.h:1321-1322)
      int64_t f = 0, z = 0;
      CBGCHK(cbg_estimate(ctx, &va, &vb, &f, &z));
      est[0] += f;
      est[1] += z;
      if (async) {
        HIPCHK(hipEventRecord(G->ev_used[t & 1], cst));
        G->used_rec[t & 1] = true;
      }
      if (st) { st->multiplies += f; st->local_ms += now_ms() - t0; ++st->stages; }
      recvA[t] = Piece();
      recvB[t] = Piece();
      continue;
    }
    cbg_csc_result C;
    int64_t m = 0;
    CBGCHK(cbg_spgemm_local(ctx, &va, &vb, sr, dt, CBG_SORTED_COLS, &C, &m));
    note_local(st, ctx, vb);
    if (async) {
      HIPCHK(hipEventRecord(G->ev_used[t & 1], cst));
      G->used_rec[t & 1] = true;
    }
    if (st) { st->multiplies += m; st->local_ms += now_ms() - t0; ++st->stages; }
    recvA[t] = Piece();   // drop references to own / received pieces
    recvB[t] = Piece();
    Piece P = piece_of_result(C);
    P.k = t % q;
    P.r = t / q;
    if (flags & CBG_RUNNING_MERGE) {
      if (acc.empty()) {
        acc.push_back(P);
      } else if (P.nnz > 0) {
        const double t1 = now_ms();
        std::vector<cbg_csc_result> two = {result_of(acc[0], dt), result_of(P, dt)};
        cbg_csc_result M;
        CBGCHK(merge_parts(ctx, two, sr, dt, &M));
        const int32_t k0 = acc[0].k, r0 = acc[0].r;
        acc.clear();
        acc.push_back(piece_of_result(M));
        acc[0].k = k0;
        acc[0].r = r0;
        if (st) st->merge_ms += now_ms() - t1;
      }
    } else if (P.nnz > 0 || parts->empty()) {
      if (!parts->empty() && (*parts)[0].nnz == 0) (*parts)[0] = P;   // keep one (empty) part only
      else parts->push_back(P);
    }
  }
  if (flags & CBG_RUNNING_MERGE) *parts = acc;
  HIPCHK(hipStreamSynchronize(G->cs));
  for (auto& e : bev) {
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e.first, e.second);
    if (st) st->bcast_ms += ms;
  }
  return CBG_OK;
}

// ------------------------------------------------------------------------------------ reduction
// Fiber all-to-all of one colsplit partial (ParFriends.h:3119-3153, Reductions.h:36-130): layer part m
// of its columns (block_range(ncol, L, m)) goes to fiber member m; returns the L pieces of this
// rank's own layer part, in member (layer) order.  The pieces own their receive storage.
//
// Values of an f64 product travel as f32 when every value of every fiber member's message survives the
// round trip f64 -> f32 -> f64 bit for bit (integers below 2^24, multiplicities, 0/1 patterns, ...): a
// lossless 1/3 cut of the bytes on the xGMI link.  Each member's verdict rides on the count exchange
// (bit 62 of its nnz), so all members agree without another collective; CBG_FIBER_NARROW=0 disables it.
cbg_status fiber_exchange(cbg_grid* G, const Piece& C, size_t vs, bool f64, std::vector<Piece>* pcs,
                          cbg_grid_stats* st) {
  cbg_ctx* ctx = G->ctx;
  hipStream_t cst = ctx->stream;
  const int L = G->L, me = G->layer;
  std::vector<int64_t> cbnd(L + 1), eb(L + 1);
  for (int m = 0; m <= L; ++m) cbnd[m] = m == L ? C.ncol : (C.ncol / L) * m;
  for (int m = 0; m <= L; ++m) HIPCHK(hipMemcpyAsync(&eb[m], C.cp + cbnd[m], 8, hipMemcpyDeviceToHost, cst));
  HIPCHK(hipStreamSynchronize(cst));
  std::vector<int64_t> snnz(L), rnnz(L);
  for (int m = 0; m < L; ++m) snnz[m] = eb[m + 1] - eb[m];
  HIPCHK(G->small.reserve(16 * (L + 1) + 16));
  int64_t* dsn = G->small.as<int64_t>();
  int64_t* drn = dsn + L;
  bool narrow = f64 && C.val != nullptr && vs == 8;
  if (narrow) {
    const char* e = std::getenv("CBG_FIBER_NARROW");
    narrow = !(e && e[0] == '0');
  }
  if (narrow) {   // does this member's whole outgoing range survive f32?
    unsigned long long* bad = (unsigned long long*)(drn + L);
    HIPCHK(hipMemsetAsync(bad, 0, 8, cst));
    const int64_t n = eb[L] - eb[0];
    if (n) k_f32_inexact<<<(int)grid_for(n, 256, kMaxGrid), 256, 0, cst>>>(n, (const double*)C.val + eb[0], bad);
    unsigned long long nb = 0;
    HIPCHK(hipMemcpyAsync(&nb, bad, 8, hipMemcpyDeviceToHost, cst));
    HIPCHK(hipStreamSynchronize(cst));
    narrow = nb == 0;
  }
  const int64_t kNarrowBit = 1LL << 62;
  std::vector<int64_t> sflag(L);
  for (int m = 0; m < L; ++m) sflag[m] = snnz[m] | (narrow ? kNarrowBit : 0);
  HIPCHK(hipMemcpyAsync(dsn, sflag.data(), 8 * L, hipMemcpyHostToDevice, cst));
  std::vector<int64_t> eight(L, 8);
  CBGCHK(t_alltoallv(G, CBG_GROUP_FIBER, dsn, eight.data(), drn, eight.data()));
  HIPCHK(hipMemcpyAsync(rnnz.data(), drn, 8 * L, hipMemcpyDeviceToHost, cst));
  HIPCHK(hipStreamSynchronize(cst));
  bool all_narrow = narrow;
  for (int m = 0; m < L; ++m) {
    all_narrow = all_narrow && (rnnz[m] & kNarrowBit);
    rnnz[m] &= ~kNarrowBit;
  }
  const int64_t myc = cbnd[me + 1] - cbnd[me];
  int64_t rtot = 0;
  for (int m = 0; m < L; ++m) rtot += rnnz[m];
  const int64_t ir_bytes = (4 * rtot + 15) & ~15LL;
  // one owner holds the received rows+values (ir) and counts (val), pieces share it
  std::shared_ptr<Owner> rx(new Owner(ctx->pool));
  StreamFence fence(cst, G->cs);
  HIPCHK(rx->ir.reserve(ir_bytes + vs * rtot + 16));
  HIPCHK(rx->val.reserve(8 * ((int64_t)L * myc + C.ncol + 2)));
  int64_t* rcnt = rx->val.as<int64_t>();
  int64_t* scnt = rcnt + (int64_t)L * myc + 1;
  char* rbase = rx->ir.as<char>();
  if (C.ncol) k_col_counts<<<(int)grid_for(C.ncol, 256, kMaxGrid), 256, 0, cst>>>(C.ncol, C.cp, scnt);
  HIPCHK(hipGetLastError());
  std::vector<int64_t> sb(L), rb(L);
  for (int m = 0; m < L; ++m) { sb[m] = 8 * (cbnd[m + 1] - cbnd[m]); rb[m] = 8 * myc; }
  CBGCHK(t_alltoallv(G, CBG_GROUP_FIBER, scnt, sb.data(), rcnt, rb.data()));
  for (int m = 0; m < L; ++m) { sb[m] = 4 * snnz[m]; rb[m] = 4 * rnnz[m]; }
  CBGCHK(t_alltoallv(G, CBG_GROUP_FIBER, C.ir + eb[0], sb.data(), rbase, rb.data()));
  const bool has_val = C.val != nullptr;
  const int64_t wire_vs = all_narrow ? 4 : (int64_t)vs;
  if (has_val && all_narrow) {   // f32 on the wire, widened back into the f64 receive region
    const int64_t stot = eb[L] - eb[0];
    PoolBuf s32, r32;
    s32.pool = r32.pool = ctx->pool;
    StreamFence fence32(cst, G->cs);
    HIPCHK(s32.reserve(4 * (stot + 1)));
    HIPCHK(r32.reserve(4 * (rtot + 1)));
    if (stot) k_f64_to_f32<<<(int)grid_for(stot, 256, kMaxGrid), 256, 0, cst>>>(stot, (const double*)C.val + eb[0],
                                                                                 s32.as<float>());
    for (int m = 0; m < L; ++m) { sb[m] = 4 * snnz[m]; rb[m] = 4 * rnnz[m]; }
    CBGCHK(t_alltoallv(G, CBG_GROUP_FIBER, s32.p, sb.data(), r32.p, rb.data()));
    if (rtot) k_f32_to_f64<<<(int)grid_for(rtot, 256, kMaxGrid), 256, 0, cst>>>(rtot, r32.as<float>(),
                                                                                (double*)(rbase + ir_bytes));
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(cst));   // s32/r32 go back to the pool on return
  } else if (has_val) {
    for (int m = 0; m < L; ++m) { sb[m] = (int64_t)vs * snnz[m]; rb[m] = (int64_t)vs * rnnz[m]; }
    CBGCHK(t_alltoallv(G, CBG_GROUP_FIBER, (const char*)C.val + vs * eb[0], sb.data(), rbase + ir_bytes, rb.data()));
  }
  if (st)
    for (int m = 0; m < L; ++m)
      if (m != me) st->fiber_bytes += (4 + (has_val ? wire_vs : 0)) * snnz[m] + 8 * (cbnd[m + 1] - cbnd[m]);
  pcs->assign(L, Piece());
  const int64_t ntiles = (myc + kScanTile - 1) / kScanTile;
  PoolBuf tiles, scal;
  tiles.pool = scal.pool = G->ctx->pool;
  HIPCHK(tiles.reserve(8 * (ntiles + 1)));
  HIPCHK(scal.reserve(16));
  int64_t off = 0;
  for (int m = 0; m < L; ++m) {
    Piece& p = (*pcs)[m];
    std::shared_ptr<Owner> o(new Owner(ctx->pool));
    HIPCHK(o->cp.reserve(8 * (myc + 1)));
    if (myc > 0) {
      k_scan_tiles<<<(int)ntiles, 256, 0, cst>>>(myc, rcnt + m * myc, tiles.as<int64_t>());
      k_scan_sums<<<1, 1024, 0, cst>>>(ntiles, tiles.as<int64_t>(), scal.as<int64_t>());
      k_scan_apply<<<(int)ntiles, 256, 0, cst>>>(myc, rcnt + m * myc, tiles.as<int64_t>(), o->cp.as<int64_t>());
    } else {
      HIPCHK(hipMemsetAsync(o->cp.p, 0, 8, cst));
    }
    p.nrow = C.nrow; p.ncol = myc; p.nnz = rnnz[m];
    p.cp = o->cp.as<int64_t>();
    p.ir = (const int32_t*)rbase + off;
    p.val = has_val ? (const void*)(rbase + ir_bytes + vs * off) : nullptr;
    p.own = o;
    p.keep = rx;
    off += rnnz[m];
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(cst));   // tiles/scal go back to the pool on return
  return CBG_OK;
}

// One chunk of the fiber message, both directions: the partial this rank sends (a chunk of the other layer's
// columns), its encoding, and the streams it receives for the same chunk of its own columns.
struct FiberMsg {
  Piece P;                                         // the sent partial
  int64_t oc = 0, n = 0;                           // its columns and entries
  int rfmt = 0, vfmt = 0;                          // rows: 0 int32, 1 16-bit gaps, 2 varint; values: 0 native,
                                                   // 1 f32, 2 u16, 3 varint
  int64_t E = 0, srow_b = 0, sesc_b = 0, sval_b = 0, svh_b = 0;
  const void* srow_p = nullptr;
  const void* sval_p = nullptr;
  const void* svh_p = nullptr;                     // the value headers (varint values) or an empty stream
  PoolBuf cpv, shdr, sval, saux, svr, svv, sescoff, svroff, svvoff, srow, sesc;
  int64_t c0 = 0, mc = 0;                          // received: my columns [c0, c0 + mc)
  int rrfmt = 0, rvfmt = 0;
  int64_t rnnz = 0, rE = 0, rrow_b = 0, rval_b = 0, rvh_b = 0;
  PoolBuf rrow, resc, rvbuf, rvhdr, rauxoff, rvoff;
  explicit FiberMsg(const std::shared_ptr<Pool>& pl) {
    for (PoolBuf* b : {&cpv, &shdr, &sval, &saux, &svr, &svv, &sescoff, &svroff, &svvoff, &srow, &sesc, &rrow, &resc,
                       &rvbuf, &rvhdr, &rauxoff, &rvoff})
      b->pool = pl;
  }
};

// exclusive scan of n int64 counts (device) into out[0..n], the total into *total (device); `tiles` is reserved by the
// caller once for the largest scan (growing a pool buffer would hand the old block back while kernels still use it)
struct Scanner {
  hipStream_t st = nullptr;
  const PoolBuf* tiles = nullptr;
  cbg_status operator()(int64_t n, const int64_t* in, int64_t* outp, int64_t* total) const {
    const int64_t nt = (n + kScanTile - 1) / kScanTile;
    if (8 * (nt + 1) > (int64_t)tiles->n) return CBG_EINVAL;
    if (n > 0) {
      k_scan_tiles<<<(int)nt, 256, 0, st>>>(n, in, tiles->as<int64_t>());
      k_scan_sums<<<1, 1024, 0, st>>>(nt, tiles->as<int64_t>(), total);
      k_scan_apply<<<(int)nt, 256, 0, st>>>(n, in, tiles->as<int64_t>(), outp);
    } else {
      HIPCHK(hipMemsetAsync(outp, 0, 8, st));
      HIPCHK(hipMemsetAsync(total, 0, 8, st));
    }
    HIPCHK(hipGetLastError());
    return CBG_OK;
  }
};

struct CodecOpts {
  bool gaps, narrow, var;
};
// CBG_FIBER_GAPS=0: int32 rows; CBG_FIBER_NARROW=0: native values; CBG_FIBER_VARINT=0: no varint codes
const CodecOpts& codec_opts() {
  static const CodecOpts o = [] {
    auto on = [](const char* n) { const char* x = std::getenv(n); return !(x && x[0] == '0'); };
    return CodecOpts{on("CBG_FIBER_GAPS"), on("CBG_FIBER_NARROW"), on("CBG_FIBER_VARINT")};
  }();
  return o;
}

// The sender's side of one fiber message (the partial m.P): one counting pass (k_code_count) gives the bytes of
// every candidate form, the message takes the smallest lossless one for its rows and for its values, and the
// encoders fill m's streams: column headers (count | aux << 32), rows, escapes, values, value headers.
// dbad: 3 device counters, dtot: 3 device totals (scratch).  Synchronises the stream once (the totals).
cbg_status fiber_encode(hipStream_t cst, const Scanner& scan, unsigned long long* dbad, int64_t* dtot, cbg_dtype dt,
                        FiberMsg& m) {
  const CodecOpts& opt = codec_opts();
  const size_t vs = dt_size(dt);
  const Piece& Po = m.P;
  m.oc = Po.ncol;
  m.n = Po.nnz;
  const int64_t oc = m.oc, n = m.n;
  const bool has_val = Po.val != nullptr;
  const bool coded = opt.gaps && oc > 0 && n > 0;
  const bool vcheck = opt.narrow && dt == CBG_F64 && has_val && vs == 8 && n > 0;
  int64_t tot[3] = {0, 0, 0};
  unsigned long long bad[3] = {0, 0, 0};
  // one pass (k_code_encode): the counts and the varint codes in per-column worst-case slots, packed below once the
  // forms are chosen; the two-pass path (k_code_count, then the encoders re-read the partial) when the slots do not
  // fit or varint codes are off (CBG_FIBER_ONEPASS=0 forces it)
  static const bool onepass_env = [] {
    const char* x = std::getenv("CBG_FIBER_ONEPASS");
    return !(x && x[0] == '0');
  }();
  int wr = 1;
  while (wr < 5 && (Po.nrow - 1) >> (7 * wr)) ++wr;   // varint bytes of the largest row (gap)
  PoolBuf slot;
  slot.pool = m.saux.pool;
  const bool onepass = coded && opt.var && onepass_env &&
                       slot.reserve((size_t)(wr + (vcheck ? 5 : 0)) * n + 16) == hipSuccess;
  if (!onepass) (void)hipGetLastError();
  uint8_t* rslot = onepass ? slot.as<uint8_t>() : nullptr;
  uint8_t* vslot = onepass && vcheck ? rslot + (int64_t)wr * n : nullptr;
  if (onepass) {
    for (PoolBuf* pb : {&m.saux, &m.svr, &m.sescoff, &m.svroff}) HIPCHK(pb->reserve(8 * (oc + 1)));
    if (vcheck) { HIPCHK(m.svv.reserve(8 * (oc + 1))); HIPCHK(m.svvoff.reserve(8 * (oc + 1))); }
    HIPCHK(hipMemsetAsync(dbad, 0, 24, cst));
    k_code_encode<<<codec_grid(oc), kCodecNT, 0, cst>>>(
        oc, Po.cp, Po.ir, vcheck ? (const double*)Po.val : nullptr, wr, rslot, vslot, m.saux.as<int64_t>(),
        m.svr.as<int64_t>(), vcheck ? m.svv.as<int64_t>() : nullptr, dbad);
    HIPCHK(hipGetLastError());
    CBGCHK(scan(oc, m.saux.as<int64_t>(), m.sescoff.as<int64_t>(), dtot + 0));
    CBGCHK(scan(oc, m.svr.as<int64_t>(), m.svroff.as<int64_t>(), dtot + 1));
    if (vcheck) CBGCHK(scan(oc, m.svv.as<int64_t>(), m.svvoff.as<int64_t>(), dtot + 2));
    HIPCHK(hipMemcpyAsync(tot, dtot, 24, hipMemcpyDeviceToHost, cst));
    HIPCHK(hipMemcpyAsync(bad, dbad, 24, hipMemcpyDeviceToHost, cst));
    HIPCHK(hipStreamSynchronize(cst));
  } else if (coded || vcheck) {
    for (PoolBuf* pb : {&m.saux, &m.svr, &m.sescoff, &m.svroff}) HIPCHK(pb->reserve(8 * (oc + 1)));
    if (vcheck) { HIPCHK(m.svv.reserve(8 * (oc + 1))); HIPCHK(m.svvoff.reserve(8 * (oc + 1))); }
    HIPCHK(hipMemsetAsync(dbad, 0, 24, cst));
    k_code_count<<<codec_grid(oc), kCodecNT, 0, cst>>>(
        oc, Po.cp, Po.ir, vcheck ? (const double*)Po.val : nullptr, m.saux.as<int64_t>(), m.svr.as<int64_t>(),
        vcheck ? m.svv.as<int64_t>() : nullptr, dbad);
    HIPCHK(hipGetLastError());
    CBGCHK(scan(oc, m.saux.as<int64_t>(), m.sescoff.as<int64_t>(), dtot + 0));
    CBGCHK(scan(oc, m.svr.as<int64_t>(), m.svroff.as<int64_t>(), dtot + 1));
    if (vcheck) CBGCHK(scan(oc, m.svv.as<int64_t>(), m.svvoff.as<int64_t>(), dtot + 2));
    HIPCHK(hipMemcpyAsync(tot, dtot, 24, hipMemcpyDeviceToHost, cst));
    HIPCHK(hipMemcpyAsync(bad, dbad, 24, hipMemcpyDeviceToHost, cst));
    HIPCHK(hipStreamSynchronize(cst));
  }
  m.rfmt = m.vfmt = 0;
  m.E = m.sesc_b = m.svh_b = 0;
  m.srow_b = 4 * n;
  if (coded && 2 * n + 4 * tot[0] < m.srow_b) { m.rfmt = 1; m.srow_b = 2 * n; m.sesc_b = 4 * tot[0]; m.E = tot[0]; }
  if (coded && opt.var && tot[1] < m.srow_b + m.sesc_b) { m.rfmt = 2; m.srow_b = tot[1]; m.sesc_b = 0; m.E = 0; }
  m.sval_b = has_val ? (int64_t)vs * n : 0;
  if (vcheck && bad[0] == 0 && 4 * n < m.sval_b) { m.vfmt = 1; m.sval_b = 4 * n; }
  if (vcheck && bad[1] == 0 && 2 * n < m.sval_b) { m.vfmt = 2; m.sval_b = 2 * n; }
  if (vcheck && opt.var && bad[2] == 0 && tot[2] + 8 * oc < m.sval_b) { m.vfmt = 3; m.sval_b = tot[2]; m.svh_b = 8 * oc; }
  m.srow_p = Po.ir;
  if (m.rfmt == 1) {
    HIPCHK(m.srow.reserve(m.srow_b + 16));
    HIPCHK(m.sesc.reserve(m.sesc_b + 16));
    k_gap_encode<<<(int)grid_for(oc, 4, kMaxGrid * 2), 256, 0, cst>>>(oc, Po.cp, Po.ir, m.sescoff.as<int64_t>(),
                                                                      m.srow.as<unsigned short>(), m.sesc.as<int32_t>());
    m.srow_p = m.srow.p;
  } else if (m.rfmt == 2) {
    HIPCHK(m.srow.reserve(m.srow_b + 16));
    if (onepass)
      k_compact_codes<<<codec_grid(oc), kCodecNT, 0, cst>>>(oc, Po.cp, wr, rslot, m.svroff.as<int64_t>(),
                                                            m.srow.as<uint8_t>());
    else
      k_var_encode<0><<<codec_grid(oc), kCodecNT, 0, cst>>>(oc, Po.cp, Po.ir, nullptr, m.svroff.as<int64_t>(),
                                                            m.srow.as<uint8_t>());
    m.srow_p = m.srow.p;
  }
  HIPCHK(m.sesc.reserve(16));   // a transport may be handed the escape buffers with zero bytes
  HIPCHK(m.shdr.reserve(8 * (oc + 1)));
  if (oc)
    k_pack_hdr<<<(int)grid_for(oc, 256, kMaxGrid), 256, 0, cst>>>(
        oc, Po.cp, m.rfmt == 1 ? m.saux.as<int64_t>() : m.rfmt == 2 ? m.svr.as<int64_t>() : nullptr,
        m.shdr.as<int64_t>());
  m.sval_p = Po.val;
  if (m.vfmt) {
    HIPCHK(m.sval.reserve(m.sval_b + 16));
    if (m.vfmt == 1)
      k_f64_to_f32<<<(int)grid_for(n, 256, kMaxGrid), 256, 0, cst>>>(n, (const double*)Po.val, m.sval.as<float>());
    else if (m.vfmt == 2)
      k_f64_to_u16<<<(int)grid_for(n, 256, kMaxGrid), 256, 0, cst>>>(n, (const double*)Po.val,
                                                                    m.sval.as<unsigned short>());
    else if (onepass)
      k_compact_codes<<<codec_grid(oc), kCodecNT, 0, cst>>>(oc, Po.cp, 5, vslot, m.svvoff.as<int64_t>(),
                                                            m.sval.as<uint8_t>());
    else
      k_var_encode<1><<<codec_grid(oc), kCodecNT, 0, cst>>>(oc, Po.cp, nullptr, (const double*)Po.val,
                                                            m.svvoff.as<int64_t>(), m.sval.as<uint8_t>());
    m.sval_p = m.sval.p;
  }
  m.svh_p = m.vfmt == 3 ? (const void*)m.svv.p : (const void*)m.sesc.p;
  HIPCHK(hipGetLastError());
  // the slots go back to the pool on return: the packing reads them first (the count exchange syncs here anyway)
  if (onepass) HIPCHK(hipStreamSynchronize(cst));
  return CBG_OK;
}

// The received streams of one message chunk (as the sender's fiber_encode made them).
struct RecvStreams {
  const void* rows;        // rrfmt 0: int32 rows, 1: u16 gaps, 2: varint gaps
  const int32_t* esc;      // rrfmt 1: escaped absolute rows
  const void* vals;        // rvfmt 0: native values, 1: f32, 2: u16, 3: varint integers
  const int64_t* vhdr;     // rvfmt 3: the columns' value bytes
};

// The receiver's side of one message chunk: m.mc columns whose absolute entry offsets are ccp[0..mc] (a scan of the
// received counts) and whose header aux (escapes / row bytes) is raux[0..mc); decodes rows into rir and values into
// rv (native type, `vs` bytes) at entries [eoff, eoff + m.rnnz).  dtot_a / dtot_v: device scratch totals.
cbg_status fiber_decode(hipStream_t cst, const Scanner& scan, int64_t* dtot_a, int64_t* dtot_v, size_t vs,
                        bool has_val, FiberMsg& m, const RecvStreams& in, const int64_t* ccp, const int64_t* raux,
                        int64_t eoff, int32_t* rir, char* rv) {
  if (m.rrfmt) {
    HIPCHK(m.rauxoff.reserve(8 * (m.mc + 1)));
    CBGCHK(scan(m.mc, raux, m.rauxoff.as<int64_t>(), dtot_a));
  }
  if (m.rnnz) {
    if (m.rrfmt == 0)
      HIPCHK(hipMemcpyAsync(rir + eoff, in.rows, 4 * m.rnnz, hipMemcpyDeviceToDevice, cst));
    else if (m.rrfmt == 1)
      k_gap_decode<<<(int)grid_for(m.mc, 4, kMaxGrid * 2), 256, 0, cst>>>(m.mc, ccp, m.rauxoff.as<int64_t>(),
                                                                           (const unsigned short*)in.rows, in.esc, rir,
                                                                           eoff);
    else
      k_var_decode<0><<<codec_grid(m.mc), kCodecNT, 0, cst>>>(m.mc, ccp, m.rauxoff.as<int64_t>(),
                                                                              (const uint8_t*)in.rows, rir, nullptr);
    if (has_val) {
      double* dv = (double*)rv;
      if (m.rvfmt == 0)
        HIPCHK(hipMemcpyAsync(rv + vs * eoff, in.vals, vs * m.rnnz, hipMemcpyDeviceToDevice, cst));
      else if (m.rvfmt == 1)
        k_f32_to_f64<<<(int)grid_for(m.rnnz, 256, kMaxGrid), 256, 0, cst>>>(m.rnnz, (const float*)in.vals, dv + eoff);
      else if (m.rvfmt == 2)
        k_u16_to_f64<<<(int)grid_for(m.rnnz, 256, kMaxGrid), 256, 0, cst>>>(m.rnnz, (const unsigned short*)in.vals,
                                                                             dv + eoff);
      else {
        HIPCHK(m.rvoff.reserve(8 * (m.mc + 1)));
        CBGCHK(scan(m.mc, in.vhdr, m.rvoff.as<int64_t>(), dtot_v));
        k_var_decode<1><<<codec_grid(m.mc), kCodecNT, 0, cst>>>(m.mc, ccp, m.rvoff.as<int64_t>(),
                                                                                (const uint8_t*)in.vals, nullptr, dv);
      }
    }
  }
  HIPCHK(hipGetLastError());
  return CBG_OK;
}

// L = 2, plain product (reduce_all_impl's exchange-after-product, overlapped): the columns of the other layer's
// part (block_range of the local columns, as fiber_exchange cuts them) are multiplied first, in C chunks of columns
// (CBG_FIBER_CHUNKS, default 2): each chunk's counts, rows and values leave for the other layer as one grouped
// ncclSend/ncclRecv on the communication stream as soon as it is made, so the link works while the next chunk and
// then the own part multiply on the compute stream; the received chunks and the own part are then merged.  The
// same two pieces and the same two-way merge as the unpipelined path, so the product is identical.  With a caller
// transport the exchange is synchronous (no overlap, same result).
//
// Wire format, per chunk and direction, each part in the smallest lossless form of the chunk (counted in one pass,
// k_code_count), announced in the count exchange (32 bytes per member: entries | formats, escapes, row bytes, value
// bytes): column headers of 8 bytes (count | aux << 32); rows as varint gaps (aux = the column's row bytes), as
// 16-bit gaps with escaped absolute rows (aux = the column's escapes) or as int32; values as varint integers (then 8
// more bytes per column: its value bytes), u16, f32 or the native f64.  A multiplicity-valued product (R-MAT A*A)
// travels at ~2-3 bytes per entry.  CBG_FIBER_GAPS=0: int32 rows; CBG_FIBER_NARROW=0: native values;
// CBG_FIBER_VARINT=0: no varint codes.

// sum over B nonzeros b of the length of A column Bir[b]: estimateFLOP of a product (mtSpGEMM.h:1117-1135), one total
__global__ void k_flops_total(int64_t nb, const int32_t* __restrict__ bir, const int64_t* __restrict__ acp,
                              unsigned long long* __restrict__ out) {
  int64_t f = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nb; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t k = bir[i];
    f += acp[k + 1] - acp[k];
  }
  f = wave_sum64(f);
  if (lane_id() == 0 && f) atomicAdd(out, (unsigned long long)f);
}

// L = 2, plain product: the fiber GATHER.  Rank (l, i, j) and its fiber partner (1-l, i, j) swap their layer operands
// instead of their partial products: each sends its A operand (the layer-l panel A(i, K_l), or its own piece when q = 1)
// and the columns of its B operand that the partner keeps (B(K_l, J_other)), receives A(i, K_{1-l}) and B(K_{1-l}, J_l),
// and multiplies A(i, [K_0 K_1]) * B([K_0; K_1], J_l) once -- the piece C(i, J_l) that the fiber reduction
// (Reductions.h:36-130, ParFriends.h:3119-3183) makes from two partials, here with no partial written twice, no codec
// and no merge.  The inner dimension is laid out in layer order on both ranks (layer 0's part first).  For A*A of a
// power-law graph the operands are ~1/100 of the partial products (s22 on 2x2x2: ~0.3 GB against ~4.8 GB coded), so the
// fiber moves far fewer bytes and the rank does the same multiplies.  Chosen by cbg_spgemm_grid when the partial's
// multiplies exceed kGatherRatio x the operand entries to send, on every rank (fiber_mode()).
constexpr double kGatherRatio = 4.0;

// the decision, agreed over the world: every rank estimates the multiplies of the half it would send as a partial
// (k_flops_total over its B operand's other columns) against the entries it would send instead, and checks that the
// gathered operands fit comfortably in free HBM
cbg_status fiber_gather_ok(cbg_grid* G, const cbg_dcsc_view& va, const cbg_dcsc_view& vb, size_t vs, bool* out) {
  cbg_ctx* ctx = G->ctx;
  hipStream_t cst = ctx->stream;
  const int other = 1 - G->layer;
  const int64_t ncol = vb.ncol;
  const int64_t cb[3] = {0, ncol / 2, ncol};
  int64_t e[2] = {0, 0};
  if (ncol > 0) {
    HIPCHK(hipMemcpyAsync(&e[0], (const int64_t*)vb.cp + cb[other], 8, hipMemcpyDeviceToHost, cst));
    HIPCHK(hipMemcpyAsync(&e[1], (const int64_t*)vb.cp + cb[other + 1], 8, hipMemcpyDeviceToHost, cst));
  }
  HIPCHK(G->small.reserve(256));
  unsigned long long* d = (unsigned long long*)G->small.as<int64_t>() + 24;
  HIPCHK(hipMemsetAsync(d, 0, 8, cst));
  HIPCHK(hipStreamSynchronize(cst));
  const int64_t nb = e[1] - e[0];
  if (nb > 0)
    k_flops_total<<<(int)grid_for(nb, 256, kMaxGrid), 256, 0, cst>>>(nb, (const int32_t*)vb.ir + e[0],
                                                                     (const int64_t*)va.cp, d);
  HIPCHK(hipGetLastError());
  unsigned long long flops = 0;
  HIPCHK(hipMemcpyAsync(&flops, d, 8, hipMemcpyDeviceToHost, cst));
  HIPCHK(hipStreamSynchronize(cst));
  const int64_t send = va.nnz + nb;
  size_t fr = 0, tot = 0;
  HIPCHK(hipMemGetInfo(&fr, &tot));
  const double bytes = 2.0 * (double)(va.nnz + vb.nnz) * (4.0 + (double)vs) * 2.0;   // received + layer-order copies
  const bool mine = (double)flops >= kGatherRatio * (double)send && bytes < 0.25 * (double)fr;
  return all_ok(G, mine, out);
}

cbg_status fiber_gather(cbg_grid* G, const cbg_dcsc_view& va, const cbg_dcsc_view& vb, cbg_semiring sr,
                        cbg_dtype dt, Piece* out, cbg_grid_stats* st) {
  cbg_ctx* ctx = G->ctx;
  hipStream_t cst = ctx->stream;
  const size_t vs = dt_size(dt);
  const int me = G->layer, other = 1 - me;
  const int64_t ncol = vb.ncol;
  const int64_t cb[3] = {0, ncol / 2, ncol};
  const double t0 = now_ms();
  // my operands as pieces: A whole; B's columns of each half (rebased colptr, arrays from the column's first entry)
  auto piece_of_view = [&](const cbg_dcsc_view& v) {
    Piece p;
    p.nrow = v.nrow; p.ncol = v.ncol; p.nnz = v.nnz;
    p.cp = (const int64_t*)v.cp; p.ir = (const int32_t*)v.ir; p.val = v.val;
    return p;
  };
  const Piece Am = piece_of_view(va);
  // A and B carry values or not independently (a pattern operand, e.g. SelectMax<bool>'s A)
  const bool hva_mine = va.val != nullptr, hvb_mine = vb.val != nullptr;
  std::shared_ptr<Owner> bo(new Owner(ctx->pool)), bm(new Owner(ctx->pool));
  auto col_piece = [&](int64_t c0, int64_t c1, Owner& o, Piece* p) -> cbg_status {
    int64_t e[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(&e[0], (const int64_t*)vb.cp + c0, 8, hipMemcpyDeviceToHost, cst));
    HIPCHK(hipMemcpyAsync(&e[1], (const int64_t*)vb.cp + c1, 8, hipMemcpyDeviceToHost, cst));
    HIPCHK(hipStreamSynchronize(cst));
    HIPCHK(o.cp.reserve(8 * (c1 - c0 + 1)));
    k_cp_rebase<<<(int)grid_for(c1 - c0 + 1, 256, kMaxGrid), 256, 0, cst>>>(c1 - c0, (const int64_t*)vb.cp, c0,
                                                                              o.cp.as<int64_t>());
    HIPCHK(hipGetLastError());
    p->nrow = vb.nrow; p->ncol = c1 - c0; p->nnz = e[1] - e[0];
    p->cp = o.cp.as<int64_t>();
    p->ir = (const int32_t*)vb.ir + e[0];
    p->val = vb.val ? (const void*)((const char*)vb.val + vs * e[0]) : nullptr;
    return CBG_OK;
  };
  Piece Bo, Bm;
  CBGCHK(col_piece(cb[other], cb[other + 1], *bo, &Bo));   // what the partner keeps
  CBGCHK(col_piece(cb[me], cb[me + 1], *bm, &Bm));         // what I keep
  // sizes: [A nrow, A ncol, A nnz, B nrow, B ncol, B nnz, has values, 0] to the partner
  HIPCHK(G->small.reserve(256));
  int64_t* dsn = G->small.as<int64_t>();
  const int64_t sz[8] = {Am.nrow, Am.ncol, Am.nnz, Bo.nrow, Bo.ncol, Bo.nnz, hva_mine ? 1 : 0, hvb_mine ? 1 : 0};
  int64_t r8[8] = {0};
  HIPCHK(hipMemcpyAsync(dsn, sz, 64, hipMemcpyHostToDevice, cst));
  int64_t segs[2] = {0, 0};
  segs[other] = 64;   // (only the partner's segment: both buffers start with it)
  CBGCHK(t_alltoallv(G, CBG_GROUP_FIBER, dsn, segs, dsn + 16, segs, G->fiber_ctl));
  HIPCHK(hipMemcpyAsync(r8, dsn + 16, 64, hipMemcpyDeviceToHost, cst));
  HIPCHK(hipStreamSynchronize(cst));
  // an operand's values travel when either side has them (an empty operand may come without a value array)
  const bool hva = hva_mine || r8[6] != 0, hvb = hvb_mine || r8[7] != 0;
  if (r8[0] != Am.nrow || r8[4] != Bm.ncol || (hva && ((Am.nnz && !Am.val) || (r8[2] && !r8[6]))) ||
      (hvb && ((Bo.nnz && !Bo.val) || (Bm.nnz && !Bm.val) || (r8[5] && !r8[7]))))
    return CBG_EDIM;
  // receive storage: the partner's A operand and B(K_other, J_me)
  std::shared_ptr<Owner> ar(new Owner(ctx->pool)), br(new Owner(ctx->pool));
  Piece Ar, Br;
  Ar.nrow = r8[0]; Ar.ncol = r8[1]; Ar.nnz = r8[2];
  Br.nrow = r8[3]; Br.ncol = r8[4]; Br.nnz = r8[5];
  for (auto* pr : {&Ar, &Br}) {
    Owner& o = pr == &Ar ? *ar : *br;
    HIPCHK(o.cp.reserve(8 * (pr->ncol + 1)));
    HIPCHK(o.ir.reserve(4 * pr->nnz + 16));
    HIPCHK(o.val.reserve(vs * pr->nnz + 16));
    pr->cp = o.cp.as<int64_t>(); pr->ir = o.ir.as<int32_t>();
    pr->val = (pr == &Ar ? hva : hvb) ? o.val.p : nullptr;
  }
  // the exchange: six arrays, each one (grouped) send/recv pair on the fiber communicator
  int64_t sent = 0;
  auto swap = [&](const void* sp, int64_t sn, void* rp, int64_t rn) -> cbg_status {
    int64_t sb[2] = {0, 0}, rb[2] = {0, 0};
    sb[other] = sn; rb[other] = rn;
    sent += sn;
    if (sn || rn) CBGCHK(t_alltoallv(G, CBG_GROUP_FIBER, sp, sb, rp, rb));
    return CBG_OK;
  };
  CBGCHK(swap(Am.cp, 8 * (Am.ncol + 1), (void*)Ar.cp, 8 * (Ar.ncol + 1)));
  CBGCHK(swap(Am.ir, 4 * Am.nnz, (void*)Ar.ir, 4 * Ar.nnz));
  if (hva) CBGCHK(swap(Am.val, (int64_t)vs * Am.nnz, (void*)Ar.val, (int64_t)vs * Ar.nnz));
  CBGCHK(swap(Bo.cp, 8 * (Bo.ncol + 1), (void*)Br.cp, 8 * (Br.ncol + 1)));
  CBGCHK(swap(Bo.ir, 4 * Bo.nnz, (void*)Br.ir, 4 * Br.nnz));
  if (hvb) CBGCHK(swap(Bo.val, (int64_t)vs * Bo.nnz, (void*)Br.val, (int64_t)vs * Br.nnz));
  const double t1 = now_ms();
  // operands in layer order: A(i, [K_0 K_1]) side by side, B([K_0; K_1], J_me) stacked by rows
  std::vector<Piece> as = me == 0 ? std::vector<Piece>{Am, Ar} : std::vector<Piece>{Ar, Am};
  std::vector<Piece> bs = me == 0 ? std::vector<Piece>{Bm, Br} : std::vector<Piece>{Br, Bm};
  Piece A2, B2;
  CBGCHK(panel_cols(ctx, as, vs, hva, &A2));
  CBGCHK(panel_rows_dt(ctx, dt, bs, hvb, &B2));
  HIPCHK(hipStreamSynchronize(cst));   // the copies are done: the received operands go back to the pool
  as.clear();
  bs.clear();
  Ar = Br = Bo = Bm = Piece();
  ar.reset(); br.reset(); bo.reset(); bm.reset();
  const cbg_dcsc_view a2 = view_of(A2, dt, hva), b2 = view_of(B2, dt, hvb);
  cbg_csc_result C;
  int64_t m = 0;
  CBGCHK(cbg_spgemm_local(ctx, &a2, &b2, sr, dt, CBG_SORTED_COLS, &C, &m));
  note_local(st, ctx, b2);
  *out = piece_of_result(C);
  out->reduced = true;
  if (st) {
    st->multiplies += m;
    st->local_ms += now_ms() - t1;
    st->fiber_bytes += sent;
    st->fiber_ms += t1 - t0;
    st->fiber_mode = 2;
  }
  return CBG_OK;
}

cbg_status fiber_pipeline(cbg_grid* G, const cbg_dcsc_view& va, const cbg_dcsc_view& vb, cbg_semiring sr,
                          cbg_dtype dt, Piece* out, cbg_grid_stats* st) {
  cbg_ctx* ctx = G->ctx;
  if (st) st->fiber_mode = 1;
  hipStream_t cst = ctx->stream;
  const size_t vs = dt_size(dt);
  const int me = G->layer, other = 1 - me;
  const int64_t ncol = vb.ncol;
  const int64_t cb[3] = {0, ncol / 2, ncol};
  const int64_t myc = cb[me + 1] - cb[me], ocw = cb[other + 1] - cb[other];
  static const int chunks_env = [] {
    const char* x = std::getenv("CBG_FIBER_CHUNKS");
    return x ? std::max(1, std::min(8, atoi(x))) : 2;
  }();
  // both members cut the columns they send (their other half = the receiver's own half) the same way
  const int C = (int)std::max<int64_t>(1, std::min<int64_t>(chunks_env, std::min(myc, ocw)));
  auto chunk = [&](int64_t w, int c, int64_t* a, int64_t* b) {
    *a = (w / C) * c;
    *b = c == C - 1 ? w : *a + w / C;
  };
  PoolBuf cpm, tiles, scal, raux;
  for (PoolBuf* b : {&cpm, &tiles, &scal, &raux}) b->pool = ctx->pool;
  // scan tiles for the largest scan, reserved once: growing a pool buffer hands the old one back to the pool while
  // kernels queued on the stream may still use it
  HIPCHK(tiles.reserve(8 * ((std::max(myc, ocw) + kScanTile - 1) / kScanTile + 1)));
  std::vector<std::unique_ptr<FiberMsg>> msgs;
  std::shared_ptr<Owner> rx(new Owner(ctx->pool));   // received headers (val), rows + values (ir)
  std::shared_ptr<Owner> co(new Owner(ctx->pool));   // the received piece's colptr
  PoolBuf dtiles, dscal;                               // the overlapped decodes' scan tiles and totals
  dtiles.pool = dscal.pool = ctx->pool;
  StreamFence fence(cst, G->cs);   // transfers into / out of the buffers above end before they return to the pool
  StreamFence dfence(G->ds);       // and so do the overlapped decodes (destroyed first: declared last)
  // columns [c0, c1) of B as a view: rebased colptr, rows and values from cp[c0]
  auto col_view = [&](int64_t c0, int64_t c1, PoolBuf& cpbuf, cbg_dcsc_view* v) -> cbg_status {
    int64_t e[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(&e[0], (const int64_t*)vb.cp + c0, 8, hipMemcpyDeviceToHost, cst));
    HIPCHK(hipMemcpyAsync(&e[1], (const int64_t*)vb.cp + c1, 8, hipMemcpyDeviceToHost, cst));
    HIPCHK(hipStreamSynchronize(cst));
    const int64_t n = c1 - c0;
    HIPCHK(cpbuf.reserve(8 * (n + 1)));
    k_cp_rebase<<<(int)grid_for(n + 1, 256, kMaxGrid), 256, 0, cst>>>(n, (const int64_t*)vb.cp, c0, cpbuf.as<int64_t>());
    HIPCHK(hipGetLastError());
    *v = vb;
    v->ncol = n; v->nzc = n; v->nnz = e[1] - e[0];
    v->cp = cpbuf.p;
    v->ir = (const int32_t*)vb.ir + e[0];
    v->val = vb.val ? (const void*)((const char*)vb.val + vs * e[0]) : nullptr;
    return CBG_OK;
  };
  const Scanner scan{cst, &tiles};
  // RCCL's kernel needs 37.6 KB of LDS per workgroup (ncclDevKernel_Generic on gfx950) and cannot share a CU with the
  // persistent heavy grid (one 1024-thread workgroup holding 152.7 KB on every CU): while a transfer is in flight the
  // products leave CBG_FIBER_RESERVE_CU CUs to it (the heavy kernels take their work from a ticket, so a workgroup held
  // back by RCCL's finds the work done instead of stretching the kernel)
  static const int reserve_env = [] {
    const char* x = std::getenv("CBG_FIBER_RESERVE_CU");
    return x ? std::max(0, atoi(x)) : kFiberReserveCu;
  }();
  const bool async = G->rccl;
  bool in_flight = false;
  HIPCHK(G->small.reserve(256));
  int64_t* dsn = G->small.as<int64_t>();   // [0..7] sent, [8..15] received, [16..18] value verdicts
  HIPCHK(scal.reserve(64));
  int64_t* dtot = scal.as<int64_t>();      // [0..2] sender totals (escapes, row bytes, value bytes), [3..5] receiver
  HIPCHK(rx->val.reserve(8 * (myc + 1)));
  int64_t* rcnt = rx->val.as<int64_t>();   // every chunk's column headers, my columns in order
  double t_local = 0, t_setup = 0;
  int64_t mults = 0;
  auto local = [&](const cbg_dcsc_view& vbx, cbg_csc_result* R, int64_t* m) -> cbg_status {
    const double t0 = now_ms();
    if (async && in_flight) ctx->reserve_cu = reserve_env;
    const cbg_status s = cbg_spgemm_local(ctx, &va, &vbx, sr, dt, CBG_SORTED_COLS, R, m);
    ctx->reserve_cu = 0;
    if (s == CBG_OK) note_local(st, ctx, vbx);
    t_local += now_ms() - t0;
    return s;
  };
  // 1. the other layer's columns, chunk by chunk: product, encoding, count exchange, transfer posted
  for (int c = 0; c < C; ++c) {
    msgs.emplace_back(new FiberMsg(ctx->pool));
    FiberMsg& m = *msgs.back();
    int64_t a, b;
    chunk(ocw, c, &a, &b);
    cbg_dcsc_view vo;
    CBGCHK(col_view(cb[other] + a, cb[other] + b, m.cpv, &vo));
    cbg_csc_result Ro;
    int64_t mo = 0;
    CBGCHK(local(vo, &Ro, &mo));
    mults += mo;
    m.P = piece_of_result(Ro);
    const double t0 = now_ms();
    CBGCHK(fiber_encode(cst, scan, (unsigned long long*)(dsn + 16), dtot, dt, m));
    const int64_t oc = m.oc, n = m.n;
    const bool has_val = m.P.val != nullptr;
    // the count exchange: [entries | rows format << 56 | values format << 58, escapes, row bytes, value bytes]
    int64_t sflag[8] = {0, 0, 0, 0, 0, 0, 0, 0}, rflag[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    sflag[4 * other + 0] = n | ((int64_t)m.rfmt << 56) | ((int64_t)m.vfmt << 58);
    sflag[4 * other + 1] = m.E;
    sflag[4 * other + 2] = m.srow_b;
    sflag[4 * other + 3] = m.sval_b;
    HIPCHK(hipMemcpyAsync(dsn, sflag, 64, hipMemcpyHostToDevice, cst));
    const int64_t thirtytwo[2] = {32, 32};
    CBGCHK(t_alltoallv(G, CBG_GROUP_FIBER, dsn, thirtytwo, dsn + 8, thirtytwo, G->fiber_ctl));
    HIPCHK(hipMemcpyAsync(rflag, dsn + 8, 64, hipMemcpyDeviceToHost, cst));
    HIPCHK(hipStreamSynchronize(cst));
    const int64_t rf = rflag[4 * other];
    m.rrfmt = (int)((rf >> 56) & 3);
    m.rvfmt = (int)((rf >> 58) & 3);
    m.rnnz = rf & ((1LL << 56) - 1);
    m.rE = rflag[4 * other + 1];
    m.rrow_b = rflag[4 * other + 2];
    m.rval_b = has_val ? rflag[4 * other + 3] : 0;
    chunk(myc, c, &m.c0, &a);
    m.mc = a - m.c0;
    m.rvh_b = m.rvfmt == 3 ? 8 * m.mc : 0;
    // receive staging of this chunk (decoded into the piece once every chunk has arrived)
    HIPCHK(m.rrow.reserve(m.rrow_b + 16));
    HIPCHK(m.resc.reserve(4 * (m.rrfmt == 1 ? m.rE : 0) + 16));
    HIPCHK(m.rvbuf.reserve(m.rval_b + 16));
    HIPCHK(m.rvhdr.reserve(m.rvh_b + 16));
    if (st) st->fiber_bytes += 8 * oc + m.srow_b + m.sesc_b + (has_val ? m.sval_b + m.svh_b : 0);
    const void* svh_p = m.svh_p;
    t_setup += now_ms() - t0;
    if (async) {
      HIPCHK(hipEventRecord(G->ev_t[0], cst));   // this chunk's headers and encoded streams are ready
      HIPCHK(hipStreamWaitEvent(G->cs, G->ev_t[0], 0));
      if (c == 0) HIPCHK(hipEventRecord(G->ev_t[1], G->cs));
      ncclComm_t f = G->comm[CBG_GROUP_FIBER];
      NCCLCHK(ncclGroupStart());
      if (oc) NCCLCHK(ncclSend(m.shdr.p, (size_t)(8 * oc), ncclInt8, other, f, G->cs));
      if (m.mc) NCCLCHK(ncclRecv(rcnt + m.c0, (size_t)(8 * m.mc), ncclInt8, other, f, G->cs));
      if (m.srow_b) NCCLCHK(ncclSend(m.srow_p, (size_t)m.srow_b, ncclInt8, other, f, G->cs));
      if (m.rrow_b) NCCLCHK(ncclRecv(m.rrow.p, (size_t)m.rrow_b, ncclInt8, other, f, G->cs));
      if (m.sesc_b) NCCLCHK(ncclSend(m.sesc.p, (size_t)m.sesc_b, ncclInt8, other, f, G->cs));
      if (m.rrfmt == 1 && m.rE) NCCLCHK(ncclRecv(m.resc.p, (size_t)(4 * m.rE), ncclInt8, other, f, G->cs));
      if (has_val && m.sval_b) NCCLCHK(ncclSend(m.sval_p, (size_t)m.sval_b, ncclInt8, other, f, G->cs));
      if (m.rval_b) NCCLCHK(ncclRecv(m.rvbuf.p, (size_t)m.rval_b, ncclInt8, other, f, G->cs));
      if (has_val && m.svh_b) NCCLCHK(ncclSend(svh_p, (size_t)m.svh_b, ncclInt8, other, f, G->cs));
      if (m.rvh_b) NCCLCHK(ncclRecv(m.rvhdr.p, (size_t)m.rvh_b, ncclInt8, other, f, G->cs));
      NCCLCHK(ncclGroupEnd());
      HIPCHK(hipEventRecord(G->ev_rx[c], G->cs));   // chunk c has arrived: the decode stream may start on it
      in_flight = true;
    } else {   // caller transport: synchronous segments (member `other` only)
      int64_t sb[2] = {0, 0}, rb[2] = {0, 0};
      auto seg = [&](const void* sp, int64_t sn, void* rp, int64_t rn) -> cbg_status {
        sb[other] = sn; rb[other] = rn;
        if (sn || rn) CBGCHK(t_alltoallv(G, CBG_GROUP_FIBER, sp, sb, rp, rb));
        return CBG_OK;
      };
      CBGCHK(seg(m.shdr.p, 8 * oc, rcnt + m.c0, 8 * m.mc));
      CBGCHK(seg(m.srow_p, m.srow_b, m.rrow.p, m.rrow_b));
      CBGCHK(seg(m.sesc.p, m.sesc_b, m.resc.p, m.rrfmt == 1 ? 4 * m.rE : 0));
      if (has_val) {
        CBGCHK(seg(m.sval_p, m.sval_b, m.rvbuf.p, m.rval_b));
        CBGCHK(seg(svh_p, m.svh_b, m.rvhdr.p, m.rvh_b));
      }
    }
  }
  if (async) HIPCHK(hipEventRecord(G->ev_t[2], G->cs));
  // 2. the received piece's storage, taken before the own product: with RCCL every chunk is decoded on the decode
  //    stream as soon as it has arrived, while the own columns multiply on the compute stream (one-wave codec
  //    workgroups fit beside the product's persistent grids and in the CUs left to the transfer).  When the storage
  //    does not fit now (or CBG_FIBER_DECODE_OVERLAP=0), the chunks are decoded after the own product, as before.
  static const bool overlap_env = [] {
    const char* x = std::getenv("CBG_FIBER_DECODE_OVERLAP");
    return !(x && x[0] == '0');
  }();
  const bool has_val = msgs.empty() || msgs[0]->P.val != nullptr;
  int64_t rnnz = 0;
  for (auto& mp : msgs) rnnz += mp->rnnz;
  const int64_t ir_bytes = (4 * rnnz + 15) & ~15LL;
  HIPCHK(co->cp.reserve(8 * (myc + 1)));
  HIPCHK(raux.reserve(8 * (myc + 1)));
  bool early = async && overlap_env && (int)msgs.size() <= 8;
  if (early) {   // only with room to spare for the own product (its output and workspace come after this)
    size_t fr = 0, tot = 0;
    HIPCHK(hipMemGetInfo(&fr, &tot));
    const double need = (double)(ir_bytes + vs * rnnz + 16);
    early = (double)fr - need >= 0.3 * (double)tot && rx->ir.reserve((size_t)need) == hipSuccess;
    if (!early) (void)hipGetLastError();
  }
  auto decode_all = [&](hipStream_t dst, const Scanner& dsc, int64_t* dt3) -> cbg_status {
    char* rbase = rx->ir.as<char>();
    int32_t* rir = (int32_t*)rbase;
    char* rv = rbase + ir_bytes;
    int64_t eoff = 0;
    for (size_t c = 0; c < msgs.size(); ++c) {
      FiberMsg& m = *msgs[c];
      if (dst != cst) HIPCHK(hipStreamWaitEvent(dst, G->ev_rx[c], 0));   // chunk c's streams and headers landed
      int64_t* ccp = co->cp.as<int64_t>() + m.c0;   // -> absolute entry offsets of the chunk's columns
      if (m.mc > 0) {
        k_split_hdr<<<(int)grid_for(m.mc, 256, kMaxGrid), 256, 0, dst>>>(m.mc, rcnt + m.c0, raux.as<int64_t>() + m.c0);
        CBGCHK(dsc(m.mc, rcnt + m.c0, ccp, dt3 + 0));
        k_add_base<<<(int)grid_for(m.mc + 1, 256, kMaxGrid), 256, 0, dst>>>(m.mc + 1, ccp, eoff);
      } else {
        HIPCHK(hipMemcpyAsync(ccp, &eoff, 8, hipMemcpyHostToDevice, dst));
        HIPCHK(hipStreamSynchronize(dst));   // (eoff lives on the host stack)
      }
      const RecvStreams in{m.rrow.p, m.resc.as<int32_t>(), m.rvbuf.p, m.rvhdr.as<int64_t>()};
      CBGCHK(fiber_decode(dst, dsc, dt3 + 1, dt3 + 2, vs, has_val, m, in, ccp, raux.as<int64_t>() + m.c0, eoff, rir,
                          rv));
      eoff += m.rnnz;
    }
    HIPCHK(hipGetLastError());
    return CBG_OK;
  };
  if (early) {
    // every buffer the overlapped decodes touch is reserved here, before any of them runs (a growing pool buffer
    // hands its old block back to the pool while queued kernels may still use it)
    HIPCHK(dtiles.reserve(8 * ((myc + kScanTile - 1) / kScanTile + 1)));
    HIPCHK(dscal.reserve(64));
    for (auto& mp : msgs) {
      HIPCHK(mp->rauxoff.reserve(8 * (mp->mc + 1)));
      HIPCHK(mp->rvoff.reserve(8 * (mp->mc + 1)));
    }
    const Scanner dscan{G->ds, &dtiles};
    CBGCHK(decode_all(G->ds, dscan, dscal.as<int64_t>()));
    HIPCHK(hipEventRecord(G->ev_t[3], G->ds));
  }
  // 3. the own columns, while the chunks travel on the communication stream (and are decoded on arrival)
  cbg_dcsc_view vm;
  CBGCHK(col_view(cb[me], cb[me + 1], cpm, &vm));
  cbg_csc_result Rm;
  int64_t mm = 0;
  CBGCHK(local(vm, &Rm, &mm));
  mults += mm;
  Piece Pm = piece_of_result(Rm);
  // 4. join; the received piece (decoded above, or now: colptr from all chunks' counts); the merge in layer order
  double t0 = now_ms();
  float xfer_ms = 0.f;
  if (async) {
    HIPCHK(hipStreamWaitEvent(cst, G->ev_t[2], 0));
    HIPCHK(hipEventSynchronize(G->ev_t[2]));
    (void)hipEventElapsedTime(&xfer_ms, G->ev_t[1], G->ev_t[2]);
  }
  if (early) {
    HIPCHK(hipStreamWaitEvent(cst, G->ev_t[3], 0));
  } else {
    if (rx->ir.reserve(ir_bytes + vs * rnnz + 16) != hipSuccess) {   // next to the two products' pieces: give the
      (void)hipGetLastError();                                        // idle product workspace back and retry once
      release_workspace(ctx);
      HIPCHK(rx->ir.reserve(ir_bytes + vs * rnnz + 16));
    }
    CBGCHK(decode_all(cst, scan, dtot + 3));
  }
  char* rbase = rx->ir.as<char>();
  int32_t* rir = (int32_t*)rbase;
  char* rv = rbase + ir_bytes;
  Piece Pr;
  Pr.nrow = Pm.nrow; Pr.ncol = myc; Pr.nnz = rnnz;
  Pr.cp = co->cp.as<int64_t>();
  Pr.ir = rir;
  Pr.val = has_val ? (const void*)rv : nullptr;
  Pr.own = co;
  Pr.keep = rx;
  HIPCHK(hipStreamSynchronize(cst));
  msgs.clear();   // the sent partials and the staging go back to the pool (the exchange has completed)
  const double t_wait = now_ms() - t0;
  t0 = now_ms();
  std::vector<cbg_csc_result> two;
  if (me == 0) two = {result_of(Pm, dt), result_of(Pr, dt)};
  else two = {result_of(Pr, dt), result_of(Pm, dt)};
  cbg_csc_result M;
  CBGCHK(merge_parts(ctx, two, sr, dt, &M));
  *out = piece_of_result(M);
  out->reduced = true;
  if (st) {
    st->multiplies += mults;
    st->local_ms += t_local;
    st->fiber_ms += t_setup + t_wait;   // exposed exchange time (the transfers themselves overlap the products)
    st->merge_ms += now_ms() - t0;
    st->fiber_xfer_ms += xfer_ms;
  }
  return CBG_OK;
}

// entries where a and b differ (bit patterns), summed into *cnt
template <typename T>
__global__ void k_count_diff(int64_t n, const T* __restrict__ a, const T* __restrict__ b,
                             unsigned long long* __restrict__ cnt) {
  int64_t c = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    c += a[i] != b[i];
  c = wave_sum64(c);
  if (lane_id() == 0 && c) atomicAdd(cnt, (unsigned long long)c);
}

// hand a piece out as a library result (move its storage when it owns it alone, else copy)
cbg_status hand_out(cbg_ctx* ctx, Piece& C, cbg_dtype dt, cbg_csc_result* out) {
  if (C.own && C.own.use_count() == 1 && !C.keep && C.cp == C.own->cp.as<int64_t>() &&
      C.ir == C.own->ir.as<int32_t>()) {
    cbg_csc_result r = result_of(C, dt);
    Owner* o = new Owner(ctx->pool);
    take(o->cp, C.own->cp);
    take(o->ir, C.own->ir);
    take(o->val, C.own->val);
    r._owner = o;
    *out = r;
    C = Piece();
    return CBG_OK;
  }
  cbg_csc_result src = result_of(C, dt);
  return cbg_col_range(ctx, &src, 0, C.ncol, out);
}

// parts -> C's colsplit piece.  Duplicates combine with SR::add in the order of the inner dimension:
// stage k, then layer l, then half r.  For every semiring but Select2nd that order is immaterial, so the
// stage products are merged first and one partial travels the fiber; Select2nd (first contributor in
// B's storage order wins, mtSpGEMM.h:583) sends every stage product and merges in (k, l, r) order, so
// the product is the same on every layout.
cbg_status reduce_all_impl(cbg_grid* G, std::vector<Piece>& parts, cbg_semiring sr, cbg_dtype dt,
                           cbg_csc_result* out, cbg_grid_stats* st) {
  cbg_ctx* ctx = G->ctx;
  const size_t vs = dt_size(dt);
  const int L = G->L;
  const bool ordered = sr == CBG_SR_SELECT2ND;
  std::stable_sort(parts.begin(), parts.end(),
                   [](const Piece& a, const Piece& b) { return a.k != b.k ? a.k < b.k : a.r < b.r; });
  auto merge_into = [&](std::vector<Piece>& ps, Piece* res) -> cbg_status {
    if (ps.size() == 1) { *res = ps[0]; return CBG_OK; }
    std::vector<cbg_csc_result> rs;
    for (auto& p : ps) rs.push_back(result_of(p, dt));
    cbg_csc_result M;
    CBGCHK(merge_parts(ctx, rs, sr, dt, &M));
    *res = piece_of_result(M);
    return CBG_OK;
  };
  Piece C;
  if (L == 1 || !ordered) {
    const double t0 = now_ms();
    CBGCHK(merge_into(parts, &C));
    parts.clear();
    if (st) st->merge_ms += now_ms() - t0;
    if (L == 1) return hand_out(ctx, C, dt, out);
    const double t1 = now_ms();
    std::vector<Piece> pcs;
    CBGCHK(fiber_exchange(G, C, vs, dt == CBG_F64, &pcs, st));
    C = Piece();
    if (st) st->fiber_ms += now_ms() - t1;
    const double t2 = now_ms();
    CBGCHK(merge_into(pcs, &C));
    pcs.clear();
    if (st) st->merge_ms += now_ms() - t2;
    return hand_out(ctx, C, dt, out);
  }
  // Select2nd on L > 1 layers: every stage product crosses the fiber on its own
  const double t1 = now_ms();
  std::vector<int32_t> ks;
  std::vector<std::vector<Piece>> got(parts.size());
  for (size_t i = 0; i < parts.size(); ++i) {
    ks.push_back(parts[i].k);
    CBGCHK(fiber_exchange(G, parts[i], vs, dt == CBG_F64, &got[i], st));
  }
  parts.clear();
  if (st) st->fiber_ms += now_ms() - t1;
  const double t2 = now_ms();
  std::vector<Piece> all;   // (k, l, r) order; parts (hence got) are sorted by (k, r)
  for (size_t i = 0; i < got.size();) {
    size_t j = i;
    while (j < got.size() && ks[j] == ks[i]) ++j;
    for (int l = 0; l < L; ++l)
      for (size_t t = i; t < j; ++t) all.push_back(got[t][l]);
    i = j;
  }
  got.clear();
  CBGCHK(merge_into(all, &C));
  all.clear();
  if (st) st->merge_ms += now_ms() - t2;
  return hand_out(ctx, C, dt, out);
}

cbg_status grid_common(cbg_ctx* ctx, int32_t world, int32_t rank, int32_t layers, int32_t rows, int32_t cols,
                       cbg_grid** out) {
  if (!ctx || !out || world <= 0 || rank < 0 || rank >= world || layers <= 0 || rows <= 0 || rows != cols ||
      layers * rows * cols != world)
    return CBG_EINVAL;
  cbg_grid* G = new cbg_grid;
  G->ctx = ctx;
  G->world = world; G->rank = rank; G->L = layers; G->q = rows;
  G->layer = rank / (rows * cols);
  G->row = (rank % (rows * cols)) / cols;
  G->col = rank % cols;
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipStreamCreateWithFlags(&G->cs, hipStreamNonBlocking));
  for (int i = 0; i < 2; ++i) {
    HIPCHK(hipEventCreateWithFlags(&G->ev_comm[i], hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&G->ev_used[i], hipEventDisableTiming));
  }
  for (int i = 0; i < 4; ++i) HIPCHK(hipEventCreate(&G->ev_t[i]));   // fiber pipeline: fences + transfer timing
  HIPCHK(hipStreamCreateWithFlags(&G->ds, hipStreamNonBlocking));
  for (hipEvent_t& e : G->ev_rx) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  *out = G;
  return CBG_OK;
}

}  // namespace

extern "C" {

cbg_status cbg_rccl_unique_id(char id[128]) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
  if (!id) return CBG_EINVAL;
  ncclUniqueId u;
  NCCLCHK(ncclGetUniqueId(&u));
  memcpy(id, &u, 128);
  return CBG_OK;
}

cbg_status cbg_grid_create_rccl(cbg_ctx* ctx, const char id[128], int32_t world, int32_t rank, int32_t layers,
                                int32_t rows, int32_t cols, cbg_grid** grid) {
  if (!id) return CBG_EINVAL;
  cbg_grid* G = nullptr;
  CBGCHK(grid_common(ctx, world, rank, layers, rows, cols, &G));
  G->rccl = true;
  ncclUniqueId u;
  memcpy(&u, id, 128);
  ncclResult_t r = ncclCommInitRank(&G->comm[CBG_GROUP_WORLD], world, u, rank);
  // sub-communicators: ROW = (layer, row) ordered by col; COL = (layer, col) by row; FIBER = (row, col) by layer
  if (r == ncclSuccess) r = ncclCommSplit(G->comm[CBG_GROUP_WORLD], G->layer * rows + G->row, G->col, &G->comm[CBG_GROUP_ROW], nullptr);
  if (r == ncclSuccess) r = ncclCommSplit(G->comm[CBG_GROUP_WORLD], G->layer * cols + G->col, G->row, &G->comm[CBG_GROUP_COL], nullptr);
  if (r == ncclSuccess) r = ncclCommSplit(G->comm[CBG_GROUP_WORLD], G->row * cols + G->col, G->layer, &G->comm[CBG_GROUP_FIBER], nullptr);
  if (r == ncclSuccess && layers > 1)
    r = ncclCommSplit(G->comm[CBG_GROUP_WORLD], G->row * cols + G->col, G->layer, &G->fiber_ctl, nullptr);
  if (r != ncclSuccess) {
    fprintf(stderr, "cbgpu: RCCL grid setup failed: %s\n", ncclGetErrorString(r));
    cbg_grid_destroy(G);
    return CBG_ECOMM;
  }
  *grid = G;
  return CBG_OK;
}

cbg_status cbg_grid_create(cbg_ctx* ctx, const cbg_transport* t, int32_t world, int32_t rank, int32_t layers,
                           int32_t rows, int32_t cols, cbg_grid** grid) {
  if (!t || !t->bcast || !t->alltoallv || !t->allgather) return CBG_EINVAL;
  cbg_grid* G = nullptr;
  CBGCHK(grid_common(ctx, world, rank, layers, rows, cols, &G));
  G->cb = *t;
  *grid = G;
  return CBG_OK;
}

cbg_status cbg_grid_destroy(cbg_grid* G) {
  if (!G) return CBG_OK;
  (void)hipSetDevice(G->ctx->device);
  if (G->cs) (void)hipStreamSynchronize(G->cs);
  for (int g = 0; g < 4; ++g)
    if (G->comm[g]) (void)ncclCommDestroy(G->comm[g]);
  if (G->fiber_ctl) (void)ncclCommDestroy(G->fiber_ctl);
  for (int i = 0; i < 2; ++i) {
    if (G->ev_comm[i]) (void)hipEventDestroy(G->ev_comm[i]);
    if (G->ev_used[i]) (void)hipEventDestroy(G->ev_used[i]);
  }
  for (int i = 0; i < 4; ++i)
    if (G->ev_t[i]) (void)hipEventDestroy(G->ev_t[i]);
  for (hipEvent_t e : G->ev_stage) (void)hipEventDestroy(e);
  if (G->cs) (void)hipStreamDestroy(G->cs);
  for (hipEvent_t e : G->ev_rx)
    if (e) (void)hipEventDestroy(e);
  if (G->ds) (void)hipStreamDestroy(G->ds);
  delete G;
  return CBG_OK;
}

cbg_status cbg_grid_query(const cbg_grid* G, cbg_grid_info* info) {
  if (!G || !info) return CBG_EINVAL;
  info->rccl = G->rccl ? 1 : 0;
  for (int g = 0; g < 4; ++g) {
    info->ranks[g] = G->gsize(g);
    if (G->rccl && G->comm[g]) {
      int n = 0;
      NCCLCHK(ncclCommCount(G->comm[g], &n));
      info->ranks[g] = n;
    }
  }
  return CBG_OK;
}

cbg_status cbg_summa_layer(cbg_grid* G, const cbg_dcsc_view* A, const cbg_dcsc_view* B, cbg_semiring sr,
                           cbg_dtype dt, uint32_t flags, cbg_csc_result* parts, int32_t* nparts,
                           cbg_grid_stats* st) {
  if (!G || !A || !B || !parts || !nparts) return CBG_EINVAL;
  HIPCHK(hipSetDevice(G->ctx->device));
  if (st) memset(st, 0, sizeof(*st));
  const double t0 = now_ms();
  std::vector<Piece> ps;
  CBGCHK(summa_layer_impl(G, A, B, sr, dt, flags & ~CBG_RUNNING_MERGE, &ps, st));
  *nparts = 0;
  for (auto& p : ps) CBGCHK(hand_out(G->ctx, p, dt, &parts[(*nparts)++]));   // stage products, stage order
  if (st) st->total_ms = now_ms() - t0;
  return CBG_OK;
}

cbg_status cbg_summa_estimate(cbg_grid* G, const cbg_dcsc_view* A, const cbg_dcsc_view* B, int64_t* flops,
                              int64_t* nnz) {
  if (!G || !A || !B || !flops || !nnz) return CBG_EINVAL;
  HIPCHK(hipSetDevice(G->ctx->device));
  std::vector<Piece> ps;
  int64_t est[2] = {0, 0};
  const cbg_dtype dt = A->val ? A->val_type : (B->val ? B->val_type : CBG_F64);
  CBGCHK(summa_layer_impl(G, A, B, CBG_SR_PLUS_TIMES, dt, 0u, &ps, nullptr, est));
  *flops = est[0];
  *nnz = est[1];
  return CBG_OK;
}

cbg_status cbg_reduce_all(cbg_grid* G, const cbg_csc_result* parts, int32_t nparts, cbg_semiring sr, cbg_dtype dt,
                          cbg_csc_result* C, cbg_grid_stats* st) {
  if (!G || !parts || nparts <= 0 || !C) return CBG_EINVAL;
  HIPCHK(hipSetDevice(G->ctx->device));
  if (st) memset(st, 0, sizeof(*st));
  const double t0 = now_ms();
  std::vector<Piece> ps(nparts);
  for (int i = 0; i < nparts; ++i) {
    ps[i].nrow = parts[i].nrow; ps[i].ncol = parts[i].ncol; ps[i].nnz = parts[i].nnz;
    ps[i].cp = parts[i].colptr; ps[i].ir = parts[i].row; ps[i].val = parts[i].val;
    ps[i].k = i;   // the stage products in stage order
  }
  CBGCHK(reduce_all_impl(G, ps, sr, dt, C, st));
  if (st) st->total_ms = now_ms() - t0;
  return CBG_OK;
}

cbg_status cbg_spgemm_grid(cbg_grid* G, const cbg_dcsc_view* A, const cbg_dcsc_view* B, cbg_semiring sr,
                           cbg_dtype dt, uint32_t flags, cbg_csc_result* C, cbg_grid_stats* st) {
  if (!G || !A || !B || !C) return CBG_EINVAL;
  HIPCHK(hipSetDevice(G->ctx->device));
  if (st) memset(st, 0, sizeof(*st));
  const double t0 = now_ms();
  std::vector<Piece> ps;
  // the panel schedule for the plain product (Mult_AnXBn_Synch / SUMMA3D); DoubleBuff / Overlap keep their
  // staged schedules, and so does Select2nd on L > 1 layers, whose fiber merge order is (stage, layer)
  const bool panels = !(flags & (CBG_HALVES | CBG_RUNNING_MERGE)) && !(sr == CBG_SR_SELECT2ND && G->L > 1) &&
                      std::getenv("CBG_GRID_STAGED") == nullptr;
  // two layers, one product per layer (panels, or one stage): the fiber exchange overlaps the product
  static const bool pipe_env = [] { const char* e = std::getenv("CBG_FIBER_PIPE"); return !(e && e[0] == '0'); }();
  const bool pipe = pipe_env && G->L == 2 && !(flags & (CBG_HALVES | CBG_RUNNING_MERGE)) && sr != CBG_SR_SELECT2ND &&
                    (panels || G->q == 1);
  CBGCHK(summa_layer_impl(G, A, B, sr, dt, flags | (panels ? kPanels : 0u) | (pipe ? kFiberPipe : 0u), &ps, st));
  if (ps.size() == 1 && ps[0].reduced) {   // the pipeline returned the reduced piece
    CBGCHK(hand_out(G->ctx, ps[0], dt, C));
  } else {
    CBGCHK(reduce_all_impl(G, ps, sr, dt, C, st));
  }
  if (st) st->total_ms = now_ms() - t0;
  return CBG_OK;
}

// The production fiber codec on one partial, without a transport (include/cbgpu.h): the chunks the pipeline would
// send, each encoded by fiber_encode and decoded by fiber_decode from the sender's own streams, then compared with
// the source chunk bit for bit.
cbg_status cbg_fiber_codec(cbg_ctx* ctx, const cbg_csc_result* P, int32_t chunks, cbg_codec_stats* out) {
  if (!ctx || !P || !out || chunks < 1) return CBG_EINVAL;
  if (P->nnz > 0 && (!P->colptr || !P->row)) return CBG_EINVAL;
  memset(out, 0, sizeof(*out));
  hipStream_t cst = ctx->stream;
  const cbg_dtype dt = P->val_type;
  const size_t vs = dt_size(dt);
  const bool has_val = P->val != nullptr;
  const int64_t ncol = P->ncol;
  const int C = (int)std::max<int64_t>(1, std::min<int64_t>(chunks, ncol));
  PoolBuf tiles, scal, cnt, hdr, raux, rcp, rbuf;
  for (PoolBuf* b : {&tiles, &scal, &cnt, &hdr, &raux, &rcp, &rbuf}) b->pool = ctx->pool;
  StreamFence fence(cst);
  HIPCHK(tiles.reserve(8 * ((ncol + kScanTile - 1) / kScanTile + 2)));
  HIPCHK(scal.reserve(128));
  HIPCHK(cnt.reserve(64));
  HIPCHK(hipMemsetAsync(cnt.p, 0, 64, cst));
  int64_t* dtot = scal.as<int64_t>();
  unsigned long long* dbad = (unsigned long long*)(dtot + 8);
  unsigned long long* dmis = cnt.as<unsigned long long>();
  const Scanner scan{cst, &tiles};
  std::vector<int64_t> hcp(ncol + 1);
  if (ncol >= 0) HIPCHK(hipMemcpyAsync(hcp.data(), P->colptr, 8 * (ncol + 1), hipMemcpyDeviceToHost, cst));
  HIPCHK(hipStreamSynchronize(cst));
  out->columns = ncol;
  out->entries = P->nnz;
  out->chunks = C;
  hipEvent_t e0 = ctx->ev[0], e1 = ctx->ev[1], e2 = ctx->ev[2];
  double enc_ms = 0, dec_ms = 0;
  for (int c = 0; c < C; ++c) {
    const int64_t a = (ncol / C) * c, b = c == C - 1 ? ncol : a + ncol / C, oc = b - a;
    FiberMsg m(ctx->pool);
    HIPCHK(m.cpv.reserve(8 * (oc + 1)));
    k_cp_rebase<<<(int)grid_for(oc + 1, 256, kMaxGrid), 256, 0, cst>>>(oc, P->colptr + a, 0, m.cpv.as<int64_t>());
    HIPCHK(hipGetLastError());
    const int64_t e_0 = hcp[a], n = hcp[b] - hcp[a];
    m.P.nrow = P->nrow; m.P.ncol = oc; m.P.nnz = n;
    m.P.cp = m.cpv.as<int64_t>();
    m.P.ir = P->row + e_0;
    m.P.val = has_val ? (const void*)((const char*)P->val + vs * e_0) : nullptr;
    HIPCHK(hipEventRecord(e0, cst));
    CBGCHK(fiber_encode(cst, scan, dbad, dtot, dt, m));
    HIPCHK(hipEventRecord(e1, cst));
    out->header_bytes += 8 * oc;
    out->row_bytes += m.srow_b;
    out->escape_bytes += m.sesc_b;
    if (has_val) { out->value_bytes += m.sval_b; out->value_header_bytes += m.svh_b; }
    if (n > 0) { out->row_formats |= 1 << m.rfmt; if (has_val) out->value_formats |= 1 << m.vfmt; }
    // the receiver's view of the same bytes: the headers split into counts + aux, the colptr a scan of the counts
    HIPCHK(hdr.reserve(8 * (oc + 1)));
    HIPCHK(raux.reserve(8 * (oc + 1)));
    HIPCHK(rcp.reserve(8 * (oc + 2)));
    const int64_t ir_bytes = (4 * n + 15) & ~15LL;
    HIPCHK(rbuf.reserve(ir_bytes + vs * n + 16));
    if (oc) HIPCHK(hipMemcpyAsync(hdr.p, m.shdr.p, 8 * oc, hipMemcpyDeviceToDevice, cst));
    if (oc) k_split_hdr<<<(int)grid_for(oc, 256, kMaxGrid), 256, 0, cst>>>(oc, hdr.as<int64_t>(), raux.as<int64_t>());
    CBGCHK(scan(oc, hdr.as<int64_t>(), rcp.as<int64_t>(), dtot + 4));
    m.rrfmt = m.rfmt; m.rvfmt = m.vfmt; m.rnnz = n; m.rE = m.E; m.mc = oc; m.c0 = 0;
    const RecvStreams in{m.srow_p, m.sesc.as<int32_t>(), m.sval_p, (const int64_t*)m.svh_p};
    int32_t* rir = rbuf.as<int32_t>();
    char* rv = rbuf.as<char>() + ir_bytes;
    CBGCHK(fiber_decode(cst, scan, dtot + 5, dtot + 6, vs, has_val, m, in, rcp.as<int64_t>(), raux.as<int64_t>(), 0,
                        rir, rv));
    HIPCHK(hipEventRecord(e2, cst));
    k_count_diff<int64_t><<<(int)grid_for(oc + 1, 256, kMaxGrid), 256, 0, cst>>>(oc + 1, rcp.as<int64_t>(),
                                                                                m.cpv.as<int64_t>(), dmis);
    if (n) {
      k_count_diff<int32_t><<<(int)grid_for(n, 256, kMaxGrid), 256, 0, cst>>>(n, rir, m.P.ir, dmis);
      if (has_val && vs == 8)
        k_count_diff<uint64_t><<<(int)grid_for(n, 256, kMaxGrid), 256, 0, cst>>>(n, (const uint64_t*)rv,
                                                                                (const uint64_t*)m.P.val, dmis);
      else if (has_val && vs == 4)
        k_count_diff<uint32_t><<<(int)grid_for(n, 256, kMaxGrid), 256, 0, cst>>>(n, (const uint32_t*)rv,
                                                                                (const uint32_t*)m.P.val, dmis);
      else if (has_val)
        k_count_diff<uint8_t><<<(int)grid_for(n, 256, kMaxGrid), 256, 0, cst>>>(n, (const uint8_t*)rv,
                                                                               (const uint8_t*)m.P.val, dmis);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(cst));   // m's buffers go back to the pool at the end of the iteration
    float t = 0.f;
    (void)hipEventElapsedTime(&t, e0, e1); enc_ms += t;
    (void)hipEventElapsedTime(&t, e1, e2); dec_ms += t;
  }
  unsigned long long mis = 0;
  HIPCHK(hipMemcpy(&mis, dmis, 8, hipMemcpyDeviceToHost));
  out->mismatches = (int64_t)mis;
  out->roundtrip_exact = mis == 0;
  out->wire_bytes = out->header_bytes + out->row_bytes + out->escape_bytes + out->value_bytes + out->value_header_bytes;
  out->encode_ms = enc_ms;
  out->decode_ms = dec_ms;
  return CBG_OK;
}

}  // extern "C"
