// abi.hip -- the C ABI of libcbgpu.so (include/cbgpu.h): contexts, staging, results, dispatch.
// Kernels and their orchestration live in spgemm_kernels.hpp / spgemm_host.hpp, instantiated per
// value dtype in inst_<dtype>.hip.
#include "spgemm_host.hpp"

// =============================================================================== C ABI
extern "C" {

int32_t cbg_abi_version(void) { return CBG_ABI_VERSION; }

const char* cbg_strerror(cbg_status s) {
  switch (s) {
    case CBG_OK: return "ok";
    case CBG_EDIM: return "dimension mismatch (DIMMISMATCH 3002)";
    case CBG_EALIAS: return "matrix alias (MATRIXALIAS 3005)";
    case CBG_ENOMEM: return "out of device memory";
    case CBG_EUNSUP: return "unsupported semiring/dtype";
    case CBG_EDEVICE: return "HIP device error or no GPU";
    case CBG_EADD: return "semiring add() called on BoolCopy1st/2nd (reference throws)";
    case CBG_EINVAL: return "invalid matrix view";
    case CBG_ECOMM: return "RCCL communication error";
  }
  return "unknown status";
}

cbg_status cbg_device_count(int32_t* n) {
  if (!n) return CBG_EINVAL;
  *n = 0;
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) return CBG_EDEVICE;
  *n = c;
  return CBG_OK;
}

cbg_status cbg_init(int device, cbg_ctx** out) {
  if (!out) return CBG_EINVAL;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0) return CBG_EDEVICE;
  HIPCHK(hipSetDevice(device));
  cbg_ctx* c = new cbg_ctx;
  c->device = device;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) { delete c; return CBG_EDEVICE; }
  c->own_stream = true;
  for (auto& e : c->ev)
    if (hipEventCreate(&e) != hipSuccess) { delete c; return CBG_EDEVICE; }
  if (hipHostMalloc(&c->pin, kPinBytes, hipHostMallocDefault) != hipSuccess) { delete c; return CBG_EDEVICE; }
  *out = c;
  return CBG_OK;
}

cbg_status cbg_destroy(cbg_ctx* c) {
  if (!c) return CBG_OK;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  for (auto& e : c->ev) if (e) (void)hipEventDestroy(e);
  if (c->pin) (void)hipHostFree(c->pin);
  if (c->own_stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return CBG_OK;
}

cbg_status cbg_set_stream(cbg_ctx* c, void* s) {
  if (!c) return CBG_EINVAL;
  if (c->own_stream) { (void)hipStreamSynchronize(c->stream); (void)hipStreamDestroy(c->stream); }
  if (s) { c->stream = (hipStream_t)s; c->own_stream = false; }
  else { HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)); c->own_stream = true; }
  return CBG_OK;
}

cbg_status cbg_synchronize(cbg_ctx* c) {
  if (!c) return CBG_EINVAL;
  HIPCHK(hipStreamSynchronize(c->stream));
  return CBG_OK;
}

cbg_status cbg_spgemm_local(cbg_ctx* ctx, const cbg_dcsc_view* A, const cbg_dcsc_view* B, cbg_semiring sr,
                            cbg_dtype out_type, uint32_t flags, cbg_csc_result* C, int64_t* multiplies_out) {
  if (!ctx || !A || !B || !C) return CBG_EINVAL;
  HIPCHK(hipSetDevice(ctx->device));
  switch (out_type) {
    case CBG_F64: return cbg_dispatch_f64(ctx, A, B, sr, flags, C, multiplies_out);
    case CBG_F32: return cbg_dispatch_f32(ctx, A, B, sr, flags, C, multiplies_out);
    case CBG_I64: return cbg_dispatch_i64(ctx, A, B, sr, flags, C, multiplies_out);
    case CBG_I32: return cbg_dispatch_i32(ctx, A, B, sr, flags, C, multiplies_out);
    case CBG_BOOL: return cbg_dispatch_b8(ctx, A, B, sr, flags, C, multiplies_out);
  }
  return CBG_EUNSUP;
}

cbg_status cbg_estimate(cbg_ctx* ctx, const cbg_dcsc_view* A, const cbg_dcsc_view* B, int64_t* mults,
                        int64_t* nnzc) {
  // the pattern product stopped after its symbolic pass and scan (kSymbolicOnly): exact multiplies and nnz(C),
  // no output formed
  cbg_dcsc_view a = *A, b = *B;
  a.val = nullptr; b.val = nullptr;
  a.val_type = b.val_type = CBG_BOOL;
  cbg_csc_result C;
  cbg_status s = cbg_spgemm_local(ctx, &a, &b, CBG_SR_PLUS_TIMES, CBG_BOOL, kSymbolicOnly, &C, mults);
  if (s != CBG_OK) return s;
  if (nnzc) *nnzc = C.nnz;
  cbg_result_free(ctx, &C);
  return CBG_OK;
}

cbg_status cbg_result_to_host(cbg_ctx* ctx, const cbg_csc_result* C, int64_t* colptr, int32_t* row, void* val) {
  if (!ctx || !C) return CBG_EINVAL;
  HIPCHK(hipSetDevice(ctx->device));
  if (colptr) HIPCHK(hipMemcpyAsync(colptr, C->colptr, sizeof(int64_t) * (C->ncol + 1), hipMemcpyDefault, ctx->stream));
  if (row && C->nnz) HIPCHK(hipMemcpyAsync(row, C->row, sizeof(int32_t) * C->nnz, hipMemcpyDefault, ctx->stream));
  if (val && C->nnz) HIPCHK(hipMemcpyAsync(val, C->val, dt_size(C->val_type) * C->nnz, hipMemcpyDefault, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return CBG_OK;
}

void cbg_result_free(cbg_ctx* ctx, cbg_csc_result* C) {
  if (!C) return;
  if (ctx) { (void)hipSetDevice(ctx->device); (void)hipStreamSynchronize(ctx->stream); }
  delete (Owner*)C->_owner;
  memset(C, 0, sizeof(*C));
}

cbg_status cbg_upload(cbg_ctx* ctx, const cbg_dcsc_view* v, cbg_csc_result* out) {
  if (!ctx || !v || !out) return CBG_EINVAL;
  const int pb = v->ptr_bytes ? v->ptr_bytes : v->idx_bytes;
  if ((v->idx_bytes != 8 && v->idx_bytes != 4) || (pb != 8 && pb != 4)) return CBG_EINVAL;
  if (v->nnz > 0 && (!v->cp || !v->ir)) return CBG_EINVAL;
  HIPCHK(hipSetDevice(ctx->device));
  std::unique_ptr<Owner> own(new Owner(ctx->pool));
  hipStream_t st = ctx->stream;
  const hipMemcpyKind kind = v->on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
  HIPCHK(own->cp.reserve(8 * (v->ncol + 1)));
  HIPCHK(own->ir.reserve(4 * (v->nnz + 1)));
  const size_t vs = v->val ? dt_size(v->val_type) : 0;
  HIPCHK(own->val.reserve(vs * (v->nnz + 1) + 8));
  DevBuf tmp;
  DevBuf tmp2;
  if (v->jc) {   // reference DCSC (cp[nzc+1], jc[nzc]) -> dense colptr on device
    const int64_t nzc = v->nzc;
    HIPCHK(tmp2.reserve(8 * (2 * nzc + 2)));
    int64_t* rcp = tmp2.as<int64_t>();
    int64_t* rjc = rcp + nzc + 1;
    DevBuf t32;
    if (pb == 8) {
      HIPCHK(hipMemcpyAsync(rcp, v->cp, 8 * (nzc + 1), kind, st));
    } else {
      HIPCHK(t32.reserve(4 * (nzc + 2)));
      HIPCHK(hipMemcpyAsync(t32.p, v->cp, 4 * (nzc + 1), kind, st));
      k_i32_to_i64<<<256, 256, 0, st>>>(nzc + 1, t32.as<int32_t>(), rcp);
      HIPCHK(hipStreamSynchronize(st));
    }
    if (v->idx_bytes == 8) {
      if (nzc) HIPCHK(hipMemcpyAsync(rjc, v->jc, 8 * nzc, kind, st));
    } else if (nzc) {
      HIPCHK(t32.reserve(4 * (nzc + 2)));
      HIPCHK(hipMemcpyAsync(t32.p, v->jc, 4 * nzc, kind, st));
      k_i32_to_i64<<<256, 256, 0, st>>>(nzc, t32.as<int32_t>(), rjc);
    }
    k_dcsc_to_csc<<<(int)grid_for(v->ncol + 1, 256, kMaxGrid), 256, 0, st>>>(v->ncol, nzc, rcp, rjc,
                                                                             own->cp.as<int64_t>());
    HIPCHK(hipStreamSynchronize(st));   // t32 is released at scope end
  } else if (pb == 8) {
    HIPCHK(hipMemcpyAsync(own->cp.p, v->cp, 8 * (v->ncol + 1), kind, st));
  } else {
    HIPCHK(tmp2.reserve(4 * (v->ncol + 2)));
    HIPCHK(hipMemcpyAsync(tmp2.p, v->cp, 4 * (v->ncol + 1), kind, st));
    k_i32_to_i64<<<256, 256, 0, st>>>(v->ncol + 1, tmp2.as<int32_t>(), own->cp.as<int64_t>());
  }
  if (v->idx_bytes == 8) {
    HIPCHK(tmp.reserve(8 * (v->nnz + 1)));
    HIPCHK(hipMemcpyAsync(tmp.p, v->ir, 8 * v->nnz, kind, st));
    k_widen_idx<<<1024, 256, 0, st>>>(v->nnz, tmp.as<int64_t>(), own->ir.as<int32_t>());
  } else {
    HIPCHK(hipMemcpyAsync(own->ir.p, v->ir, 4 * v->nnz, kind, st));
  }
  if (v->val && v->nnz) HIPCHK(hipMemcpyAsync(own->val.p, v->val, vs * v->nnz, kind, st));
  HIPCHK(hipStreamSynchronize(st));
  memset(out, 0, sizeof(*out));
  out->nrow = v->nrow; out->ncol = v->ncol; out->nnz = v->nnz;
  out->colptr = own->cp.as<int64_t>(); out->row = own->ir.as<int32_t>();
  out->val = v->val ? own->val.p : nullptr;
  out->val_type = v->val_type;
  out->_owner = own.release();
  return CBG_OK;
}

cbg_status cbg_result_view(const cbg_csc_result* C, cbg_dcsc_view* v) {
  if (!C || !v) return CBG_EINVAL;
  memset(v, 0, sizeof(*v));
  v->nrow = C->nrow; v->ncol = C->ncol; v->nnz = C->nnz; v->nzc = C->ncol;
  v->cp = C->colptr; v->jc = nullptr; v->ir = C->row; v->idx_bytes = 4; v->ptr_bytes = 8;
  v->val = C->val; v->val_type = C->val_type; v->on_device = 1;
  return CBG_OK;
}

cbg_status cbg_last_profile(cbg_ctx* ctx, cbg_profile* p) {
  if (!ctx || !p) return CBG_EINVAL;
  *p = ctx->prof;
  return CBG_OK;
}

}  // extern "C"

extern "C" cbg_status cbg_merge(cbg_ctx* ctx, const cbg_csc_result* parts, int32_t nparts, cbg_semiring sr,
                                cbg_dtype val_type, uint32_t flags, cbg_csc_result* C) {
  if (!ctx || !parts || nparts <= 0 || !C) return CBG_EINVAL;
  HIPCHK(hipSetDevice(ctx->device));
  switch (val_type) {
    case CBG_F64: return cbg_merge_f64(ctx, parts, nparts, sr, flags, C);
    case CBG_F32: return cbg_merge_f32(ctx, parts, nparts, sr, flags, C);
    case CBG_I64: return cbg_merge_i64(ctx, parts, nparts, sr, flags, C);
    case CBG_I32: return cbg_merge_i32(ctx, parts, nparts, sr, flags, C);
    case CBG_BOOL: return cbg_merge_b8(ctx, parts, nparts, sr, flags, C);
  }
  return CBG_EUNSUP;
}
