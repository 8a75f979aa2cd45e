// pybind11 entry points for the HIP kernel library (module fleetx_amd._C._kernels).
// Tensors cross the boundary as raw device addresses (uintptr_t) plus the
// current HIP stream handle; shape checks live in fleetx_amd/ops/*.py.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <stdint.h>
#include <string>
#include <stdexcept>
#include <vector>

namespace py = pybind11;
typedef uintptr_t ptr;

extern "C" {
int fx_coltile_splits(int rows, int cols);
void fx_add_ln_fwd(int, const void*, const void*, const void*, const void*, const void*, void*,
                   void*, float*, float*, int, int, float, float, uint64_t, hipStream_t);
void fx_ln_bwd_row(int, const void*, const void*, const float*, const float*, const void*,
                   const void*, void*, void*, int, int, float, uint64_t, hipStream_t);
int fx_ln_bwd_cols_blocks(int, int, int);
int fx_ln_bwd_cols(int, const void*, const void*, const float*, const float*, const void*,
                   const void*, void*, void*, int, int, float, uint64_t, float*, int, float*, void*,
                   int, float*, void*, int, float*, void*, int, hipStream_t);
void fx_coltile_partial(int, int, const void*, const void*, const float*, const float*, float*,
                        float*, int, int, int, hipStream_t, int*, float*, void*, int, float*,
                        void*, int);
void fx_coltile_finalize(int, const float*, int, int, float*, void*, int, hipStream_t);
void fx_bias_gelu_fwd(int, int, const void*, const void*, void*, long, int, hipStream_t);
void fx_bias_gelu_bwd(int, int, const void*, const void*, const void*, void*, float*, int, int, int,
                      hipStream_t, int*, float*, void*, int);
void fx_bias_dropout_add_fwd(int, const void*, const void*, const void*, void*, long, int, float,
                             uint64_t, hipStream_t);
void fx_dropout_bwd_colsum(int, const void*, void*, float*, int, int, int, float, uint64_t,
                           hipStream_t, int*, float*, void*, int);
void fx_dropout_fwd(int, const void*, void*, long, float, uint64_t, hipStream_t);
void fx_ce_stats(int, const void*, const int64_t*, int, int, long, float*, float*, float*, int,
                 hipStream_t);
void fx_ce_bwd(int, const void*, void*, const int64_t*, const float*, const float*, int, int, long,
               int, hipStream_t);
int fx_sumsq_blocks(long n);
void fx_sumsq_f32(const float*, long, float*, int, hipStream_t);
void fx_sumsq_16(int, const void*, long, float*, int, hipStream_t);
void fx_sumsq_chunks(const int64_t*, const int64_t*, int, float*, hipStream_t);
void fx_adamw_tune(int, int, int);
void fx_adamw_flat(int, float*, const float*, float*, float*, void*, long, float, float, float,
                   float, float, float, const float*, const int*, const int*, hipStream_t);
void fx_adamw_flat_g16(int, float*, const void*, float*, float*, void*, long, float, float,
                       float, float, float, float, const float*, const int*, const int*,
                       hipStream_t);
int fx_adamw_flat_pk(int, void*, const void*, float*, float*, void*, long, float, float, float,
                     float, float, float, const float*, const int*, const int*, hipStream_t);
int fx_adamw_flat_pk_g16(int, void*, const void*, float*, float*, void*, long, float, float,
                         float, float, float, float, const float*, const int*, const int*,
                         hipStream_t);
void fx_pk_split(const float*, void*, void*, long, hipStream_t);
void fx_pk_join(const void*, const void*, float*, long, hipStream_t);
void fx_cast_f32(int, const float*, void*, long, hipStream_t);
void fx_accum_f32(int, float*, const void*, long, int, hipStream_t);
void fx_embedding_fwd(int, const int64_t*, const int64_t*, const void*, const void*, void*, int,
                      int, long, long, hipStream_t);
void fx_embedding_bwd(int, const int64_t*, const void*, float*, int, int, long, long,
                      hipStream_t);
void fx_fa_set_dkdv64(int);
void fx_fa_set_dq64(int);
void fx_fa_set_dkdv_vreg(int);
int fx_fa_lab();
int fx_fa_set_stamps(void*);
int fx_flash_fwd(int, const void*, const void*, const void*, void*, float*, const long*, const long*,
                 const long*, const long*, const int*, const float*, long, int, int, int, int, int,
                 int, float, float, uint64_t, hipStream_t);
int fx_flash_bwd(int, const void*, const void*, const void*, const void*, const void*, const float*,
                 float*, void*, void*, void*, const long*, const long*, const long*, const long*,
                 const long*, const long*, const int*, const float*, long, int, int, int, int, int,
                 int, float, float, uint64_t, hipStream_t);
int fx_fake_quant_fwd(int, const void*, void*, const float*, int, long, hipStream_t);
void fx_absmax(int, const void*, long, float*, hipStream_t);
int fx_gn_nseg(long, long);
int fx_gn_fwd(int, const void*, const float*, const float*, const float*, const float*, void*,
              double*, float*, float*, int, int, int, long, int, float, int, hipStream_t);
int fx_gn_bwd_reduce(int, const void*, const void*, const float*, const float*, const float*,
                     const float*, const float*, const float*, float*, int, int, int, long, int,
                     int, hipStream_t);
int fx_gn_bwd_apply(int, const void*, const void*, const float*, const float*, const float*,
                    const float*, const float*, const float*, const float*, const float*, void*,
                    int, int, int, long, int, int, hipStream_t);
int fx_transpose16(int, const void*, void*, float*, int, int, long, long, hipStream_t);
int fx_sample(int, const void*, long, int, int, float, int, float, const float*, int64_t*, float*,
              float*, hipStream_t);
int fx_decode_attn(int, const void*, const void*, const void*, void*, const int*, int, int, int,
                   int, int, float*, long, long, long, long, long, long, float, hipStream_t);
void fx_embedding_bwd_sorted(int, const int64_t*, const int64_t*, const void*, float*, int, int,
                             long, long, hipStream_t);
int fx_softmax_fwd(int, int, const void*, const void*, void*, long, int, int, long, float, int,
                   hipStream_t);
int fx_softmax_bwd(int, const void*, const void*, void*, long, int, int, float, int, hipStream_t);
int fx_gemm(int, int, int, int, int, int, int, const void*, long, const void*, long, void*, long,
            const void*, void*, long, int, hipStream_t, float*, float*);
long fx_gemm_ws_bytes(int, int, int, int);
void fx_gemm_set_gm(int);
void fx_gemm_set_geom(int, int);
int fx_gemm_tuned(long*, int);
void fx_gemm_set_tuned(int, int, int, int, int, int, int);
void fx_gemm_set_tune(int);
void fx_gemm_set_persist(int);
void fx_gemm_set_xrect(int);
int fx_decode_gemv(int, int, int, int, int, const void*, long, const void*, long, const void*,
                   const void*, long, void*, long, void*, void*, const long*, int, int, int,
                   const void*, const void*, float, hipStream_t);
void fx_set_dropout_salt(const void*);
hipStream_t fx_cumask_stream_create(int, int*);
int fx_stream_destroy(hipStream_t);
void fx_set_adamw_lr_ptr(const void*);
int fx_comm_max_world();
int fx_comm_max_blocks();
void* fx_comm_alloc(long);
int fx_comm_free(void*);
int fx_comm_ipc_handle(void*, char*);
void* fx_comm_ipc_open(const char*);
int fx_comm_ipc_close(void*);
int fx_comm_allreduce(int, int, const void*, void*, long, int, int, const uint64_t*, unsigned int*,
                      unsigned int*, long, unsigned long long, hipStream_t);
}

#define P(x) reinterpret_cast<void*>(x)
#define CP(x) reinterpret_cast<const void*>(x)
#define S(x) reinterpret_cast<hipStream_t>(x)
#define F(x) reinterpret_cast<float*>(x)

static std::vector<long> v3(const std::vector<long>& a) {
  std::vector<long> r(a);
  r.resize(3, 0);
  return r;
}

PYBIND11_MODULE(_kernels, m) {
  m.doc() = "FleetX-AMD HIP kernels (gfx950)";
  m.def("coltile_splits", &fx_coltile_splits);
  m.def("add_ln_fwd", [](int dt, ptr x, ptr bias, ptr res, ptr g, ptr b, ptr s_out, ptr y,
                         ptr mean, ptr rstd, int rows, int h, float eps, float p, uint64_t key,
                         ptr st) {
    fx_add_ln_fwd(dt, CP(x), CP(bias), CP(res), CP(g), CP(b), P(s_out), P(y), F(mean), F(rstd),
                  rows, h, eps, p, key, S(st));
  });
  m.def("ln_bwd_row", [](int dt, ptr dy, ptr s, ptr mean, ptr rstd, ptr g, ptr ds_in, ptr ds_out,
                         ptr dx_out, int rows, int h, float p, uint64_t key, ptr st) {
    fx_ln_bwd_row(dt, CP(dy), CP(s), F(mean), F(rstd), CP(g), CP(ds_in), P(ds_out), P(dx_out),
                  rows, h, p, key, S(st));
  });
  // LayerNorm backward with dgamma / dbeta (/ dbias of the fused residual's
  // linear) column sums in the same pass; returns -1 if h is not covered
  m.def("ln_bwd_cols_blocks", &fx_ln_bwd_cols_blocks);
  m.def("ln_bwd_cols", [](int dt, ptr dy, ptr s, ptr mean, ptr rstd, ptr g, ptr ds_in, ptr ds_out,
                          ptr dx_out, int rows, int h, float p, uint64_t key, ptr part,
                          int with_dbias, ptr fg, ptr tg, int accg, ptr fb, ptr tb, int accb,
                          ptr fx, ptr tx, int accx, ptr st) {
    return fx_ln_bwd_cols(dt, CP(dy), CP(s), F(mean), F(rstd), CP(g), CP(ds_in), P(ds_out),
                          P(dx_out), rows, h, p, key, F(part), with_dbias, F(fg), P(tg), accg,
                          F(fb), P(tb), accb, F(fx), P(tx), accx, S(st));
  }, py::arg("dt"), py::arg("dy"), py::arg("s"), py::arg("mean"), py::arg("rstd"), py::arg("g"),
     py::arg("ds_in"), py::arg("ds_out"), py::arg("dx_out"), py::arg("rows"), py::arg("h"),
     py::arg("p"), py::arg("key"), py::arg("part"), py::arg("with_dbias"), py::arg("fg") = 0,
     py::arg("tg") = 0, py::arg("accg") = 0, py::arg("fb") = 0, py::arg("tb") = 0,
     py::arg("accb") = 0, py::arg("fx") = 0, py::arg("tx") = 0, py::arg("accx") = 0,
     py::arg("st") = 0);
  // column-sum producers: cnt != 0 fuses the finalize (last workgroup of a
  // column tile sums the splits into f*/t* outputs); cnt == 0: the caller
  // runs coltile_finalize
  m.def("coltile_partial", [](int dt, int mode, ptr a, ptr b, ptr mean, ptr rstd, ptr p0, ptr p1,
                              int rows, int cols, int splits, ptr st, ptr cnt, ptr f0, ptr t0,
                              int acc0, ptr f1, ptr t1, int acc1) {
    fx_coltile_partial(dt, mode, CP(a), CP(b), F(mean), F(rstd), F(p0), F(p1), rows, cols, splits,
                       S(st), reinterpret_cast<int*>(cnt), F(f0), P(t0), acc0, F(f1), P(t1),
                       acc1);
  }, py::arg("dt"), py::arg("mode"), py::arg("a"), py::arg("b"), py::arg("mean"), py::arg("rstd"),
     py::arg("p0"), py::arg("p1"), py::arg("rows"), py::arg("cols"), py::arg("splits"),
     py::arg("st"), py::arg("cnt") = 0, py::arg("f0") = 0, py::arg("t0") = 0, py::arg("acc0") = 0,
     py::arg("f1") = 0, py::arg("t1") = 0, py::arg("acc1") = 0);
  m.def("coltile_finalize", [](int dt, ptr part, int splits, int cols, ptr out_f32, ptr out_t,
                               int accumulate, ptr st) {
    fx_coltile_finalize(dt, F(part), splits, cols, F(out_f32), P(out_t), accumulate, S(st));
  });
  m.def("bias_gelu_fwd", [](int dt, int erf, ptr x, ptr bias, ptr y, long n, int cols, ptr st) {
    fx_bias_gelu_fwd(dt, erf, CP(x), CP(bias), P(y), n, cols, S(st));
  });
  m.def("bias_gelu_bwd", [](int dt, int erf, ptr dy, ptr x, ptr bias, ptr dx, ptr part, int rows,
                            int cols, int splits, ptr st, ptr cnt, ptr out_f32, ptr out_t,
                            int acc) {
    fx_bias_gelu_bwd(dt, erf, CP(dy), CP(x), CP(bias), P(dx), F(part), rows, cols, splits, S(st),
                     reinterpret_cast<int*>(cnt), F(out_f32), P(out_t), acc);
  }, py::arg("dt"), py::arg("erf"), py::arg("dy"), py::arg("x"), py::arg("bias"), py::arg("dx"),
     py::arg("part"), py::arg("rows"), py::arg("cols"), py::arg("splits"), py::arg("st"),
     py::arg("cnt") = 0, py::arg("out_f32") = 0, py::arg("out_t") = 0, py::arg("acc") = 0);
  m.def("bias_dropout_add_fwd", [](int dt, ptr x, ptr bias, ptr res, ptr out, long n, int cols,
                                   float p, uint64_t key, ptr st) {
    fx_bias_dropout_add_fwd(dt, CP(x), CP(bias), CP(res), P(out), n, cols, p, key, S(st));
  });
  m.def("dropout_bwd_colsum", [](int dt, ptr dout, ptr dx, ptr part, int rows, int cols,
                                 int splits, float p, uint64_t key, ptr st, ptr cnt, ptr out_f32,
                                 ptr out_t, int acc) {
    fx_dropout_bwd_colsum(dt, CP(dout), P(dx), F(part), rows, cols, splits, p, key, S(st),
                          reinterpret_cast<int*>(cnt), F(out_f32), P(out_t), acc);
  }, py::arg("dt"), py::arg("dout"), py::arg("dx"), py::arg("part"), py::arg("rows"),
     py::arg("cols"), py::arg("splits"), py::arg("p"), py::arg("key"), py::arg("st"),
     py::arg("cnt") = 0, py::arg("out_f32") = 0, py::arg("out_t") = 0, py::arg("acc") = 0);
  m.def("dropout_fwd", [](int dt, ptr x, ptr y, long n, float p, uint64_t key, ptr st) {
    fx_dropout_fwd(dt, CP(x), P(y), n, p, key, S(st));
  });
  m.def("ce_stats", [](int dt, ptr logits, ptr labels, int rows, int V, long vstart, ptr mx,
                       ptr sm, ptr tg, int ignore, ptr st) {
    fx_ce_stats(dt, CP(logits), reinterpret_cast<const int64_t*>(labels), rows, V, vstart, F(mx),
                F(sm), F(tg), ignore, S(st));
  });
  m.def("ce_bwd", [](int dt, ptr logits, ptr dx, ptr labels, ptr lse, ptr g, int rows, int V,
                     long vstart, int ignore, ptr st) {
    fx_ce_bwd(dt, CP(logits), P(dx), reinterpret_cast<const int64_t*>(labels), F(lse), F(g), rows,
              V, vstart, ignore, S(st));
  });
  m.def("sumsq_blocks", &fx_sumsq_blocks);
  m.def("sumsq_chunks", [](ptr addr, ptr len, int n, ptr partial, ptr st) {
    fx_sumsq_chunks(reinterpret_cast<const int64_t*>(addr), reinterpret_cast<const int64_t*>(len),
                    n, F(partial), S(st));
  });
  m.def("sumsq_f32", [](ptr x, long n, ptr partial, int blocks, ptr st) {
    fx_sumsq_f32(F(x), n, F(partial), blocks, S(st));
  });
  m.def("sumsq_16", [](int dt, ptr x, long n, ptr partial, int blocks, ptr st) {
    fx_sumsq_16(dt, CP(x), n, F(partial), blocks, S(st));
  });
  m.def("adamw_tune", &fx_adamw_tune, py::arg("grid"), py::arg("nt"), py::arg("wide") = 0);
  m.def("adamw_flat", [](int dt, ptr p, ptr g, ptr mm, ptr vv, ptr p16, long n, float lr,
                         float b1, float b2, float eps, float wd, float l2, ptr gscale, ptr skip,
                         ptr step, ptr st) {
    fx_adamw_flat(dt, F(p), F(g), F(mm), F(vv), P(p16), n, lr, b1, b2, eps, wd, l2, F(gscale),
                  reinterpret_cast<const int*>(skip), reinterpret_cast<const int*>(step), S(st));
  });
  m.def("adamw_flat_g16", [](int dt, ptr p, ptr g, ptr mm, ptr vv, ptr p16, long n, float lr,
                             float b1, float b2, float eps, float wd, float l2, ptr gscale,
                             ptr skip, ptr step, ptr st) {
    fx_adamw_flat_g16(dt, F(p), CP(g), F(mm), F(vv), P(p16), n, lr, b1, b2, eps, wd, l2,
                      F(gscale), reinterpret_cast<const int*>(skip),
                      reinterpret_cast<const int*>(step), S(st));
  });
  // packed master: p = the master's low halves, p16 = the bf16 parameters (high halves)
  m.def("adamw_flat_pk", [](int dt, ptr p, ptr g, ptr mm, ptr vv, ptr p16, long n, float lr,
                            float b1, float b2, float eps, float wd, float l2, ptr gscale,
                            ptr skip, ptr step, ptr st) {
    return fx_adamw_flat_pk(dt, P(p), CP(g), F(mm), F(vv), P(p16), n, lr, b1, b2, eps, wd, l2,
                            F(gscale), reinterpret_cast<const int*>(skip),
                            reinterpret_cast<const int*>(step), S(st));
  });
  m.def("adamw_flat_pk_g16", [](int dt, ptr p, ptr g, ptr mm, ptr vv, ptr p16, long n, float lr,
                                float b1, float b2, float eps, float wd, float l2, ptr gscale,
                                ptr skip, ptr step, ptr st) {
    return fx_adamw_flat_pk_g16(dt, P(p), CP(g), F(mm), F(vv), P(p16), n, lr, b1, b2, eps, wd,
                                l2, F(gscale), reinterpret_cast<const int*>(skip),
                                reinterpret_cast<const int*>(step), S(st));
  });
  m.def("pk_split", [](ptr x, ptr hi, ptr lo, long n, ptr st) {
    fx_pk_split(F(x), P(hi), P(lo), n, S(st));
  });
  m.def("pk_join", [](ptr hi, ptr lo, ptr x, long n, ptr st) {
    fx_pk_join(CP(hi), CP(lo), F(x), n, S(st));
  });
  m.def("cast_f32", [](int dt, ptr x, ptr y, long n, ptr st) {
    fx_cast_f32(dt, F(x), P(y), n, S(st));
  });
  m.def("accum_f32", [](int dt, ptr acc, ptr x, long n, int overwrite, ptr st) {
    fx_accum_f32(dt, F(acc), CP(x), n, overwrite, S(st));
  });
  m.def("embedding_fwd", [](int dt, ptr ids, ptr pos, ptr W, ptr Pw, ptr out, int ntok, int h,
                            long vstart, long vsize, ptr st) {
    fx_embedding_fwd(dt, reinterpret_cast<const int64_t*>(ids),
                     reinterpret_cast<const int64_t*>(pos), CP(W), CP(Pw), P(out), ntok, h, vstart,
                     vsize, S(st));
  });
  m.def("embedding_bwd", [](int dt, ptr ids, ptr dout, ptr dW, int ntok, int h, long vstart,
                            long vsize, ptr st) {
    fx_embedding_bwd(dt, reinterpret_cast<const int64_t*>(ids), CP(dout), F(dW), ntok, h, vstart,
                     vsize, S(st));
  });
  m.def("embedding_bwd_sorted", [](int dt, ptr sid, ptr perm, ptr dout, ptr dW, int ntok, int h,
                                   long vstart, long vsize, ptr st) {
    fx_embedding_bwd_sorted(dt, reinterpret_cast<const int64_t*>(sid),
                            reinterpret_cast<const int64_t*>(perm), CP(dout), F(dW), ntok, h,
                            vstart, vsize, S(st));
  });
  m.def("fa_set_dkdv64", &fx_fa_set_dkdv64);
  m.def("fa_set_dq64", &fx_fa_set_dq64);
  m.def("fa_set_dkdv_vreg", &fx_fa_set_dkdv_vreg);
  m.def("fa_set_stamps", [](ptr p) { return fx_fa_set_stamps(P(p)); });  // lab builds: fwd stamps
  m.def("fa_lab", &fx_fa_lab);  // 1 in tools/fa_lab builds (lab attention variants)
  m.def("flash_fwd", [](int dt, ptr q, ptr k, ptr v, ptr out, ptr lse, std::vector<long> qs,
                        std::vector<long> ks, std::vector<long> vs, std::vector<long> os,
                        ptr kv_lens, ptr kbias, long kb_stride, int B, int H, int Sq, int Sk, int D,
                        int causal, float scale, float p, uint64_t key, ptr st) {
    auto a = v3(qs), b = v3(ks), c = v3(vs), d = v3(os);
    return fx_flash_fwd(dt, CP(q), CP(k), CP(v), P(out), F(lse), a.data(), b.data(), c.data(),
                        d.data(), reinterpret_cast<const int*>(kv_lens), F(kbias), kb_stride, B, H,
                        Sq, Sk, D, causal, scale, p, key, S(st));
  });
  m.def("flash_bwd", [](int dt, ptr q, ptr k, ptr v, ptr o, ptr dout, ptr lse, ptr delta, ptr dq,
                        ptr dk,
                        ptr dv, std::vector<long> qs, std::vector<long> ks, std::vector<long> vs,
                        std::vector<long> os, std::vector<long> dqs, std::vector<long> dks,
                        ptr kv_lens, ptr kbias, long kb_stride, int B, int H, int Sq, int Sk, int D,
                        int causal, float scale, float p, uint64_t key, ptr st) {
    auto a = v3(qs), b = v3(ks), c = v3(vs), d = v3(os), e = v3(dks), f = v3(dqs);
    return fx_flash_bwd(dt, CP(q), CP(k), CP(v), CP(o), CP(dout), F(lse), F(delta), P(dq), P(dk),
                        P(dv), a.data(), b.data(), c.data(), d.data(), f.data(), e.data(),
                        reinterpret_cast<const int*>(kv_lens), F(kbias), kb_stride, B, H, Sq, Sk,
                        D, causal, scale, p, key, S(st));
  });
  m.def("gn_nseg", [](long rows, long hw) { return fx_gn_nseg(rows, hw); });
  m.def("gn_fwd", [](int dt, ptr x, ptr gamma, ptr beta, ptr scale, ptr shift, ptr y, ptr part,
                     ptr mean, ptr rstd, int B, int C, int G, long hw, int nseg, float eps,
                     int silu, ptr st) {
    return fx_gn_fwd(dt, CP(x), F(gamma), F(beta), F(scale), F(shift), P(y),
                     reinterpret_cast<double*>(part), F(mean), F(rstd), B, C, G, hw, nseg, eps,
                     silu, S(st));
  });
  m.def("gn_bwd_reduce", [](int dt, ptr x, ptr dy, ptr mean, ptr rstd, ptr gamma, ptr beta,
                            ptr scale, ptr shift, ptr part, int B, int C, int G, long hw, int nseg,
                            int silu, ptr st) {
    return fx_gn_bwd_reduce(dt, CP(x), CP(dy), F(mean), F(rstd), F(gamma), F(beta), F(scale),
                            F(shift), F(part), B, C, G, hw, nseg, silu, S(st));
  });
  m.def("gn_bwd_apply", [](int dt, ptr x, ptr dy, ptr mean, ptr rstd, ptr gamma, ptr beta,
                           ptr scale, ptr shift, ptr g1, ptr g2, ptr dx, int B, int C, int G,
                           long hw, int nseg, int silu, ptr st) {
    return fx_gn_bwd_apply(dt, CP(x), CP(dy), F(mean), F(rstd), F(gamma), F(beta), F(scale),
                           F(shift), F(g1), F(g2), P(dx), B, C, G, hw, nseg, silu, S(st));
  });
  m.def("fake_quant_fwd", [](int dt, ptr x, ptr y, ptr scale, int bits, long n, ptr st) {
    return fx_fake_quant_fwd(dt, CP(x), P(y), F(scale), bits, n, S(st));
  });
  m.def("absmax", [](int dt, ptr x, long n, ptr out, ptr st) {
    fx_absmax(dt, CP(x), n, F(out), S(st));
  });
  m.def("transpose16", [](int dt, ptr x, ptr y, ptr part, int R, int C, long ldx, long ldy,
                          ptr st) { return fx_transpose16(dt, CP(x), P(y), F(part), R, C, ldx, ldy, S(st)); });
  m.def("sample", [](int dt, ptr logits, long ld, int B, int V, float inv_temp, int top_k,
                     float top_p, ptr u, ptr ids, ptr lse, ptr probs, ptr st) {
    return fx_sample(dt, CP(logits), ld, B, V, inv_temp, top_k, top_p, F(u),
                     reinterpret_cast<int64_t*>(ids), F(lse), F(probs), S(st));
  });
  m.def("decode_attn", [](int dt, ptr q, ptr kc, ptr vc, ptr out, ptr lens, int B, int H, int D,
                          int maxlen, int nsplit, ptr ws, long sqb, long sqh, long skb, long sks,
                          long skh, long sob, float scale, ptr st) {
    return fx_decode_attn(dt, CP(q), CP(kc), CP(vc), P(out), reinterpret_cast<const int*>(lens), B,
                          H, D, maxlen, nsplit, F(ws), sqb, sqh, skb, sks, skh, sob, scale, S(st));
  });
  m.def("softmax_fwd", [](int dt, int mdt, ptr x, ptr mask, ptr y, long rows, int Sq, int Sk,
                          long mask_div, float scale, int causal, ptr st) {
    return fx_softmax_fwd(dt, mdt, CP(x), CP(mask), P(y), rows, Sq, Sk, mask_div, scale, causal,
                          S(st));
  });
  m.def("gemm", [](int dt, int la, int lb, int epi, int M, int N, int K, ptr A, long lda, ptr B,
                   long ldb, ptr C, long ldc, ptr bias, ptr aux, long ldaux, int beta, ptr st,
                   ptr sq, ptr ws) {
    return fx_gemm(dt, la, lb, epi, M, N, K, CP(A), lda, CP(B), ldb, P(C), ldc, CP(bias), P(aux),
                   ldaux, beta, S(st), F(sq), F(ws));
  }, py::arg("dt"), py::arg("la"), py::arg("lb"), py::arg("epi"), py::arg("M"), py::arg("N"),
     py::arg("K"), py::arg("A"), py::arg("lda"), py::arg("B"), py::arg("ldb"), py::arg("C"),
     py::arg("ldc"), py::arg("bias"), py::arg("aux"), py::arg("ldaux"), py::arg("beta"),
     py::arg("st"), py::arg("sq") = 0, py::arg("ws") = 0);
  m.def("gemm_ws_bytes", &fx_gemm_ws_bytes);
  m.def("gemm_set_gm", &fx_gemm_set_gm);
  m.def("gemm_set_geom", &fx_gemm_set_geom);
  m.def("gemm_set_tuned", &fx_gemm_set_tuned);
  m.def("gemm_set_tune", &fx_gemm_set_tune);
  m.def("gemm_set_persist", &fx_gemm_set_persist);
  m.def("gemm_set_xrect", &fx_gemm_set_xrect);
  m.def("gemm_tuned", []() {
    std::vector<long> buf(7 * 512);
    const int n = fx_gemm_tuned(buf.data(), (int)buf.size());
    py::list rows;
    for (int i = 0; i < n; ++i)
      rows.append(py::make_tuple(buf[7 * i], buf[7 * i + 1], buf[7 * i + 2], buf[7 * i + 3],
                                 buf[7 * i + 4], buf[7 * i + 5], buf[7 * i + 6]));
    return rows;
  });
  // decode-time skinny GEMM with fused sub-layer epilogues (decode_gemv.hip)
  m.def("decode_gemv", [](int dt, int epi, int M, int N, int K, ptr x, long ldx, ptr w, long ldw,
                          ptr bias, ptr res, long ldres, ptr y, long ldy, ptr kc, ptr vc, ptr pos,
                          int heads, int head_dim, int maxlen, ptr ln_w, ptr ln_b, float ln_eps,
                          ptr st) {
    return fx_decode_gemv(dt, epi, M, N, K, CP(x), ldx, CP(w), ldw, CP(bias), CP(res), ldres, P(y),
                          ldy, P(kc), P(vc), reinterpret_cast<const long*>(pos), heads, head_dim,
                          maxlen, CP(ln_w), CP(ln_b), ln_eps, S(st));
  });
  // CU-masked stream (streams.hip): returns (stream handle, CUs selected)
  m.def("cumask_stream_create", [](int ncu) {
    int got = 0;
    hipStream_t s = fx_cumask_stream_create(ncu, &got);
    return py::make_tuple(reinterpret_cast<ptr>(s), got);
  });
  m.def("stream_destroy", [](ptr s) { return fx_stream_destroy(S(s)); });
  // graph mode: device-resident dropout salt / AdamW learning rate (0 = off)
  m.def("set_dropout_salt", [](ptr p) { fx_set_dropout_salt(CP(p)); });
  m.def("set_adamw_lr_ptr", [](ptr p) { fx_set_adamw_lr_ptr(CP(p)); });
  // intra-node one-shot all-reduce over IPC-mapped peer memory (comm.hip)
  m.def("comm_max_world", &fx_comm_max_world);
  m.def("comm_max_blocks", &fx_comm_max_blocks);
  m.def("comm_alloc", [](long slot_granules) {
    return reinterpret_cast<ptr>(fx_comm_alloc(slot_granules));
  });
  m.def("comm_free", [](ptr p) { return fx_comm_free(P(p)); });
  m.def("comm_ipc_handle", [](ptr p) {
    char h[64];
    const int r = fx_comm_ipc_handle(P(p), h);
    if (r != 0) throw std::runtime_error("hipIpcGetMemHandle failed: " + std::to_string(r));
    return py::bytes(h, 64);
  });
  m.def("comm_ipc_open", [](py::bytes h) {
    std::string s = h;
    if (s.size() != 64) throw std::runtime_error("IPC handle must be 64 bytes");
    return reinterpret_cast<ptr>(fx_comm_ipc_open(s.data()));
  });
  m.def("comm_ipc_close", [](ptr p) { return fx_comm_ipc_close(P(p)); });
  m.def("comm_allreduce", [](int dt, int op, ptr in, ptr out, long n, int rank, int world,
                             std::vector<uint64_t> peers, ptr epochs, ptr err, long slot,
                             unsigned long long timeout_ticks, ptr st) {
    if ((int)peers.size() != world) throw std::runtime_error("need one receive base per rank");
    return fx_comm_allreduce(dt, op, CP(in), P(out), n, rank, world, peers.data(),
                             reinterpret_cast<unsigned int*>(epochs),
                             reinterpret_cast<unsigned int*>(err), slot, timeout_ticks, S(st));
  });
  m.def("softmax_bwd", [](int dt, ptr y, ptr dy, ptr dx, long rows, int Sq, int Sk, float scale,
                          int causal, ptr st) {
    return fx_softmax_bwd(dt, CP(y), CP(dy), P(dx), rows, Sq, Sk, scale, causal, S(st));
  });
}
