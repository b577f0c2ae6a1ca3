// torch <-> HIP kernel bindings for llm_weighted_consensus_amd.ops._kernels.
// Every op: validates device/dtype/shape on the host (a kernel must never see operands whose shape
// disagrees with its grid), then launches on the caller's current HIP stream so it can be captured
// into a hipGraph by torch.cuda.CUDAGraph.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

extern "C" {
int lwc_rmsnorm(const void*, void*, const void*, void*, int, int, float, hipStream_t);
int lwc_rmsnorm_quant_fp8(const void*, void*, const void*, void*, int, int, float, void*, float*, hipStream_t);
int lwc_layernorm(const void*, const void*, const void*, const void*, const void*, void*, int, int, float, hipStream_t);
int lwc_rope_kv_write(void*, const int*, const int*, const float*, const float*, void*, void*, int, int, int, int,
                      int, int, hipStream_t);
int lwc_silu_mul(const void*, void*, int, int, int, hipStream_t);
int lwc_embedding_gather(const void*, const int*, void*, int, int, int, hipStream_t);
int lwc_kv_block_copy(void*, const int*, int, int, int, long long, hipStream_t);
int lwc_kv_gather(const void*, const void*, const long long*, void*, void*, int, int, int, int, hipStream_t);
int lwc_paged_decode(const void*, int, const void*, const void*, const int*, const int*, void*, float*, float*, int,
                     int, int, int, int, int, int, float, const float*, const float*, const int*, hipStream_t);
int lwc_set_decode_wave_min_items(int);
int lwc_paged_decode_cascade(const void*, int, const void*, const void*, const int*, const int*, const int*, int, void*,
                             int, int, int, int, int, float, const float*, const float*, const int*, void*, void*, int, hipStream_t);
int lwc_cascade_rows_per_tile(int);
int lwc_grouped_gemm(const void*, const void*, void*, const int*, const float*, const float*, const void*, const int*,
                     int, int, int, int, int, int, long long, int, float*, int, long long, hipStream_t);
int lwc_gemm8p(const void*, const void*, void*, const void*, float*, int*, int, int, int, int, int, int, hipStream_t);
int lwc_gemm8p_slots();
int lwc_gemm4w(const void*, const void*, void*, const void*, int, int, int, int, int, int, int, float*, int, int, int,
               float, int, int, int, int, float*, int*, hipStream_t);
int lwc_rms_rowsumsq(const void*, float*, int, int, hipStream_t);
int lwc_skinny_gemm(const void*, const void*, void*, const void*, int, int, int, int, int, int, hipStream_t);
int lwc_gemm8g_fp8(const void*, const void*, void*, const int*, const int*, const float*, const float*, int, int, int,
                   int, int, int, int, int, int, const void*, void*, int, hipStream_t);
int lwc_moe_route(const void*, int, int, int, int*, float*, int*, int*, int*, hipStream_t);
int lwc_moe_router(const void*, int, const void*, int, int, int, int, int*, float*, int*, int*, int*, void*,
                   hipStream_t);
int lwc_moe_combine(const void*, const int*, const float*, int, int, int, void*, hipStream_t);
int lwc_quant_fp8_rows(const void*, int, int, void*, float*, hipStream_t);
int lwc_ep_pack(const void*, const float*, const int*, const int*, int, int, int, int, int, void*, hipStream_t);
int lwc_ep_unpack(const void*, int, int, int, int, int, int, void*, float*, int*, int*, hipStream_t);
int lwc_ep_back(const void*, const int*, int, int, int, void*, hipStream_t);
int lwc_ep_combine(const void*, const int*, const int*, const float*, int, int, int, int, int, int, void*, hipStream_t);
int lwc_silu_mul_quant_fp8(const void*, int, int, int, void*, float*, hipStream_t);
int lwc_prefill_attention(const void*, const void*, const void*, void*, const int*, const int*, int, int, int, int, int, int, int,
                          int, int, float, int, hipStream_t);
int lwc_prefill_attention_mx(const void*, const void*, const void*, void*, void*, int, const int*, int, int, int, int,
                             int, int, int, int, float, int, hipStream_t);
int lwc_prefill_attention_paged(const void*, const void*, const void*, void*, const int*, const int*, const int*, int, int,
                                int, int, int, int, int, int, float, hipStream_t);
int lwc_sample(const void*, int, int, int, const float*, const float*, const int*, const float*, const float*,
               const float*, const float*, const float*, void*, const int*, const float*, const int*,
               const unsigned int*, const int*, const unsigned long long*, const unsigned long long*, int, int,
               int, int*, float*, int*, float*, hipStream_t);
long long lwc_ar_region_bytes(int, long long);
int lwc_ar_alloc(long long, void**, void*);
int lwc_ar_open(const void*, void**);
int lwc_ar_close(void*);
int lwc_ar_free(void*);
int lwc_ar_handle_bytes();
int lwc_allreduce(void* const*, int, int, const void*, void*, long long, long long, int*, int, long long, hipStream_t);
int lwc_alltoall(void* const*, int, int, const void*, void*, long long, long long, int*, int, long long, hipStream_t);
int lwc_pool_l2norm(const void*, int, const int*, int, int, int, float*, void*, hipStream_t);
int lwc_cosine_consensus(const void*, int, int, int, float*, float, float*, float*, int*, hipStream_t);
int lwc_knn_topk(const float*, int, int, const float*, int, float*, int*, float*, int*, hipStream_t);
int lwc_vote_tally(const double*, const double*, const unsigned char*, int, int, int, double*, double*, double*,
                   hipStream_t);
}

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

// V cache of one layer: [NB, Hkv, BS/4, D, 4] bf16, the 4-token interleaved layout of the decode kernels.
void check_v_cache(const at::Tensor& v, const at::Tensor& k, const char* who) {
  TORCH_CHECK(v.dim() == 5 && v.size(0) == k.size(0) && v.size(1) == k.size(1) && v.size(2) * 4 == k.size(2) &&
                  v.size(3) == k.size(3) && v.size(4) == 4 && v.is_contiguous(),
              who, ": v_cache must be [NB, Hkv, BS/4, D, 4] matching k_cache [NB, Hkv, BS, D]");
}

#define CHECK_GPU(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_DTYPE(t, dt) TORCH_CHECK((t).scalar_type() == (dt), #t " has dtype ", (t).scalar_type(), ", expected ", dt)
#define CHECK_BF16(t) \
  CHECK_GPU(t);       \
  CHECK_DTYPE(t, at::kBFloat16)
#define CHECK_RC(rc, name) TORCH_CHECK((rc) == 0, name " launch failed with code ", (rc))

template <typename T>
const T* opt_ptr(const c10::optional<at::Tensor>& t) {
  return t.has_value() && t->defined() ? reinterpret_cast<const T*>(t->data_ptr()) : nullptr;
}

void rmsnorm(const at::Tensor& x, const c10::optional<at::Tensor>& residual, const at::Tensor& w, at::Tensor& out,
             double eps) {
  CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out);
  CHECK_CONTIG(x); CHECK_CONTIG(out);
  const int d = (int)x.size(-1);
  const int rows = (int)(x.numel() / std::max<int64_t>(d, 1));
  TORCH_CHECK(w.numel() == d && out.numel() == x.numel(), "rmsnorm: shape mismatch");
  void* r = nullptr;
  if (residual.has_value() && residual->defined()) {
    CHECK_BF16(*residual); CHECK_CONTIG(*residual);
    TORCH_CHECK(residual->numel() == x.numel(), "rmsnorm: residual shape mismatch");
    r = residual->data_ptr();
  }
  CHECK_RC(lwc_rmsnorm(x.data_ptr(), r, w.data_ptr(), out.data_ptr(), rows, d, (float)eps, cur_stream()), "rmsnorm");
}

void rmsnorm_quant_fp8(const at::Tensor& x, const c10::optional<at::Tensor>& residual, const at::Tensor& w,
                       const c10::optional<at::Tensor>& out, at::Tensor& q, at::Tensor& scale, double eps) {
  // K1 + K11e: RMSNorm (+ residual update) whose output is also quantised per row to e4m3 (q, scale);
  // out (the bf16 output) is optional.  d in {2048, 4096, 8192}.
  CHECK_BF16(x); CHECK_BF16(w); CHECK_CONTIG(x); CHECK_GPU(q); CHECK_CONTIG(q); CHECK_CONTIG(scale);
  CHECK_DTYPE(scale, at::kFloat);
  TORCH_CHECK(q.scalar_type() == at::kFloat8_e4m3fn, "rmsnorm_quant_fp8: q must be e4m3fn");
  const int d = (int)x.size(-1);
  const int rows = (int)(x.numel() / std::max<int64_t>(d, 1));
  TORCH_CHECK(d == 2048 || d == 4096 || d == 8192, "rmsnorm_quant_fp8: d must be 2048, 4096 or 8192");
  TORCH_CHECK(w.numel() == d && q.numel() == x.numel() && scale.numel() >= rows, "rmsnorm_quant_fp8: shape mismatch");
  void* r = nullptr;
  if (residual.has_value() && residual->defined()) {
    CHECK_BF16(*residual); CHECK_CONTIG(*residual);
    TORCH_CHECK(residual->numel() == x.numel(), "rmsnorm_quant_fp8: residual shape mismatch");
    r = residual->data_ptr();
  }
  void* y = nullptr;
  if (out.has_value() && out->defined()) {
    CHECK_BF16(*out); CHECK_CONTIG(*out);
    TORCH_CHECK(out->numel() == x.numel(), "rmsnorm_quant_fp8: out shape mismatch");
    y = out->data_ptr();
  }
  CHECK_RC(lwc_rmsnorm_quant_fp8(x.data_ptr(), r, w.data_ptr(), y, rows, d, (float)eps, q.data_ptr(),
                                 scale.data_ptr<float>(), cur_stream()),
           "rmsnorm_quant_fp8");
}

void layernorm(const at::Tensor& x, const c10::optional<at::Tensor>& residual, const at::Tensor& g,
               const at::Tensor& b, at::Tensor& out, double eps, const c10::optional<at::Tensor>& pre_bias) {
  CHECK_BF16(x); CHECK_BF16(g); CHECK_BF16(b); CHECK_BF16(out);
  CHECK_CONTIG(x); CHECK_CONTIG(out);
  const int d = (int)x.size(-1);
  const int rows = (int)(x.numel() / std::max<int64_t>(d, 1));
  TORCH_CHECK(g.numel() == d && b.numel() == d && out.numel() == x.numel(), "layernorm: shape mismatch");
  const void* r = nullptr;
  if (residual.has_value() && residual->defined()) {
    CHECK_BF16(*residual); CHECK_CONTIG(*residual);
    TORCH_CHECK(residual->numel() == x.numel(), "layernorm: residual shape mismatch");
    r = residual->data_ptr();
  }
  const void* pb = nullptr;
  if (pre_bias.has_value() && pre_bias->defined()) {
    CHECK_BF16(*pre_bias); CHECK_CONTIG(*pre_bias);
    TORCH_CHECK(pre_bias->numel() == d, "layernorm: pre-norm bias shape mismatch");
    pb = pre_bias->data_ptr();
  }
  CHECK_RC(lwc_layernorm(x.data_ptr(), r, pb, g.data_ptr(), b.data_ptr(), out.data_ptr(), rows, d, (float)eps,
                         cur_stream()),
           "layernorm");
}

void rope_kv_write(at::Tensor& qkv, const at::Tensor& positions, const c10::optional<at::Tensor>& slots,
                   const at::Tensor& cos_t, const at::Tensor& sin_t, at::Tensor& k_cache, at::Tensor& v_cache,
                   int64_t Hq, int64_t Hkv, int64_t D, bool rope_q) {
  CHECK_BF16(qkv); CHECK_CONTIG(qkv);
  CHECK_GPU(positions); CHECK_DTYPE(positions, at::kInt);
  CHECK_DTYPE(cos_t, at::kFloat); CHECK_DTYPE(sin_t, at::kFloat);
  CHECK_BF16(k_cache); CHECK_BF16(v_cache);
  const int T = (int)qkv.size(0);
  TORCH_CHECK(qkv.size(1) == (Hq + 2 * Hkv) * D, "rope_kv_write: qkv row is not (Hq+2Hkv)*D");
  TORCH_CHECK(positions.numel() == T, "rope_kv_write: positions length");
  TORCH_CHECK(cos_t.size(1) == D / 2 && sin_t.size(1) == D / 2, "rope_kv_write: cos/sin table width");
  // k_cache [NB, Hkv, BS, D]; v_cache [NB, Hkv, BS/4, D, 4] (4-token interleaved)
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(1) == Hkv && k_cache.size(3) == D, "rope_kv_write: k_cache shape");
  check_v_cache(v_cache, k_cache, "rope_kv_write");
  const int BS = (int)k_cache.size(2);
  const int* sp = nullptr;
  if (slots.has_value() && slots->defined()) {
    CHECK_DTYPE(*slots, at::kInt);
    TORCH_CHECK(slots->numel() == T, "rope_kv_write: slots length");
    sp = slots->data_ptr<int>();
  }
  CHECK_RC(lwc_rope_kv_write(qkv.data_ptr(), positions.data_ptr<int>(), sp, cos_t.data_ptr<float>(),
                             sin_t.data_ptr<float>(), k_cache.data_ptr(), v_cache.data_ptr(), T, (int)Hq, (int)Hkv,
                             (int)D, BS, rope_q ? 1 : 0, cur_stream()),
           "rope_kv_write");
}

// Optional q rotation inside the decode kernels: (cos [max_pos, D/2] fp32, sin, positions [B] int32) all
// given or none.
struct QRope {
  const float* cos = nullptr;
  const float* sin = nullptr;
  const int* pos = nullptr;
};
static QRope q_rope(const c10::optional<at::Tensor>& c, const c10::optional<at::Tensor>& s,
                    const c10::optional<at::Tensor>& pos, int B, int D, const char* what) {
  QRope r;
  const bool any = (c.has_value() && c->defined()) || (s.has_value() && s->defined()) ||
                   (pos.has_value() && pos->defined());
  if (!any) return r;
  TORCH_CHECK(c.has_value() && s.has_value() && pos.has_value() && c->defined() && s->defined() && pos->defined(),
              what, ": rope needs cos, sin and positions");
  CHECK_DTYPE(*c, at::kFloat); CHECK_DTYPE(*s, at::kFloat); CHECK_DTYPE(*pos, at::kInt);
  CHECK_CONTIG(*c); CHECK_CONTIG(*s); CHECK_CONTIG(*pos);
  TORCH_CHECK(c->dim() == 2 && c->size(1) == D / 2 && s->sizes() == c->sizes(), what, ": rope table shape");
  TORCH_CHECK(pos->numel() >= B, what, ": positions shorter than the batch");
  r.cos = c->data_ptr<float>();
  r.sin = s->data_ptr<float>();
  r.pos = pos->data_ptr<int>();
  return r;
}

void silu_mul(const at::Tensor& in, at::Tensor& out, int64_t block) {
  CHECK_BF16(in); CHECK_BF16(out); CHECK_CONTIG(in); CHECK_CONTIG(out);
  const int F = (int)out.size(-1);
  const int T = (int)(out.numel() / std::max(F, 1));
  TORCH_CHECK(in.size(-1) == 2 * F && in.numel() == 2 * out.numel(), "silu_mul: shape mismatch");
  TORCH_CHECK(block == 0 || (block % 8 == 0 && F % block == 0), "silu_mul: block must divide F, multiple of 8");
  CHECK_RC(lwc_silu_mul(in.data_ptr(), out.data_ptr(), T, F, (int)block, cur_stream()), "silu_mul");
}

void embedding(const at::Tensor& table, const at::Tensor& ids, at::Tensor& out) {
  CHECK_BF16(table); CHECK_BF16(out); CHECK_CONTIG(table); CHECK_CONTIG(out);
  CHECK_GPU(ids); CHECK_DTYPE(ids, at::kInt);
  const int T = (int)ids.numel(), d = (int)table.size(1);
  TORCH_CHECK(out.numel() == (int64_t)T * d, "embedding: out shape");
  CHECK_RC(lwc_embedding_gather(table.data_ptr(), ids.data_ptr<int>(), out.data_ptr(), T, d, (int)table.size(0),
                                cur_stream()),
           "embedding");
}

void kv_gather(const at::Tensor& kc, const at::Tensor& vc, const at::Tensor& slots, at::Tensor& ko, at::Tensor& vo) {
  // kc [NB, Hkv, BS, D], vc [NB, Hkv, BS/4, D, 4] (one layer), slots [n] int64 (< NB*BS, checked by the
  // caller's block manager), ko/vo [n, Hkv*D] contiguous bf16
  CHECK_BF16(kc); CHECK_BF16(vc); CHECK_BF16(ko); CHECK_BF16(vo); CHECK_CONTIG(kc); CHECK_CONTIG(vc);
  CHECK_DTYPE(slots, at::kLong); CHECK_CONTIG(slots); CHECK_CONTIG(ko); CHECK_CONTIG(vo);
  TORCH_CHECK(kc.dim() == 4 && vc.dim() == 5, "kv_gather: cache layouts");
  const int Hkv = (int)kc.size(1), BS = (int)kc.size(2), D = (int)kc.size(3);
  const int n = (int)slots.numel();
  TORCH_CHECK(ko.size(0) == n && vo.size(0) == n && ko.size(1) == Hkv * D && vo.size(1) == Hkv * D,
              "kv_gather: output shapes");
  CHECK_RC(lwc_kv_gather(kc.data_ptr(), vc.data_ptr(), (const long long*)slots.data_ptr<int64_t>(), ko.data_ptr(),
                         vo.data_ptr(), n, Hkv, D, BS, cur_stream()),
           "kv_gather");
}

void kv_block_copy(at::Tensor& cache, const at::Tensor& pairs) {
  // cache: [L*2, NB, ...block...]
  CHECK_BF16(cache); CHECK_CONTIG(cache);
  CHECK_GPU(pairs); CHECK_DTYPE(pairs, at::kInt); CHECK_CONTIG(pairs);
  TORCH_CHECK(pairs.dim() == 2 && pairs.size(1) == 2, "kv_block_copy: pairs must be [P, 2]");
  const int LK = (int)cache.size(0), NB = (int)cache.size(1);
  const long long be = cache.numel() / ((long long)LK * NB);
  CHECK_RC(lwc_kv_block_copy(cache.data_ptr(), pairs.data_ptr<int>(), (int)pairs.size(0), LK, NB, be, cur_stream()),
           "kv_block_copy");
}

void paged_decode(const at::Tensor& q, const at::Tensor& k_cache, const at::Tensor& v_cache,
                  const at::Tensor& block_tables, const at::Tensor& ctx_lens, at::Tensor& out,
                  const c10::optional<at::Tensor>& part_o, const c10::optional<at::Tensor>& part_lse,
                  int64_t num_splits, double scale, const c10::optional<at::Tensor>& rope_cos,
                  const c10::optional<at::Tensor>& rope_sin, const c10::optional<at::Tensor>& positions) {
  // q: [B, >= Hq*D] with row stride; out: [B, Hq, D]
  CHECK_BF16(q); CHECK_BF16(k_cache); CHECK_BF16(v_cache); CHECK_BF16(out);
  CHECK_DTYPE(block_tables, at::kInt); CHECK_DTYPE(ctx_lens, at::kInt);
  CHECK_CONTIG(block_tables); CHECK_CONTIG(ctx_lens); CHECK_CONTIG(out);
  TORCH_CHECK(q.stride(-1) == 1, "paged_decode: q rows must be contiguous");
  const int B = (int)out.size(0), Hq = (int)out.size(1), D = (int)out.size(2);
  const int Hkv = (int)k_cache.size(1), BS = (int)k_cache.size(2);
  TORCH_CHECK(q.size(0) == B && q.size(1) >= Hq * D, "paged_decode: q shape");
  check_v_cache(v_cache, k_cache, "paged_decode");
  TORCH_CHECK(block_tables.size(0) == B && ctx_lens.numel() == B, "paged_decode: batch mismatch");
  float* po = nullptr;
  float* pl = nullptr;
  if (num_splits > 1) {
    TORCH_CHECK(part_o.has_value() && part_lse.has_value(), "paged_decode: split-K needs workspaces");
    TORCH_CHECK(part_o->numel() >= (int64_t)B * Hq * num_splits * D && part_lse->numel() >= (int64_t)B * Hq * num_splits,
                "paged_decode: workspace too small");
    po = part_o->data_ptr<float>();
    pl = part_lse->data_ptr<float>();
  }
  const QRope qr = q_rope(rope_cos, rope_sin, positions, B, D, "paged_decode");
  CHECK_RC(lwc_paged_decode(q.data_ptr(), (int)q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                            block_tables.data_ptr<int>(), ctx_lens.data_ptr<int>(), out.data_ptr(), po, pl, B, Hq, Hkv,
                            D, BS, (int)block_tables.size(1), (int)num_splits, (float)scale, qr.cos, qr.sin, qr.pos,
                            cur_stream()),
           "paged_decode");
}

void paged_decode_cascade(const at::Tensor& q, const at::Tensor& k_cache, const at::Tensor& v_cache,
                          const at::Tensor& block_tables, const at::Tensor& ctx_lens, const at::Tensor& tiles,
                          const c10::optional<at::Tensor>& out, int64_t Hq, double scale,
                          const c10::optional<at::Tensor>& rope_cos, const c10::optional<at::Tensor>& rope_sin,
                          const c10::optional<at::Tensor>& positions, const c10::optional<at::Tensor>& out8,
                          const c10::optional<at::Tensor>& mx) {
  // tiles: [max_tiles, 3] int32 super-tiles (row_start, nseq, prefix_blocks), nseq <= cascade_rows_per_tile(G);
  // the engine builds them on the host (rows must stay < B: the kernel trusts the table).
  // out8 + mx instead of out: e4m3 rows [B, Hq * D] with e8m0 scales [Hq, >= B, 4] (one per 32 dims of a head)
  CHECK_BF16(q); CHECK_BF16(k_cache); CHECK_BF16(v_cache);
  const bool mxo = out8.has_value() && out8->defined();
  TORCH_CHECK(mxo == (mx.has_value() && mx->defined()), "paged_decode_cascade: out8 and mx go together");
  TORCH_CHECK(mxo || (out.has_value() && out->defined()), "paged_decode_cascade: out or out8 + mx");
  check_v_cache(v_cache, k_cache, "paged_decode_cascade");
  CHECK_DTYPE(block_tables, at::kInt); CHECK_DTYPE(ctx_lens, at::kInt); CHECK_DTYPE(tiles, at::kInt);
  CHECK_CONTIG(tiles); CHECK_CONTIG(block_tables); CHECK_CONTIG(ctx_lens);
  TORCH_CHECK(tiles.dim() == 2 && tiles.size(1) == 3, "paged_decode_cascade: tiles must be [T, 3]");
  TORCH_CHECK(q.dim() == 2 && q.stride(1) == 1, "paged_decode_cascade: q must be [B, >=Hq*D] rows");
  const int B = (int)q.size(0), D = (int)k_cache.size(3), Hkv = (int)k_cache.size(1), BS = (int)k_cache.size(2);
  TORCH_CHECK(block_tables.size(0) >= B && ctx_lens.numel() >= B, "paged_decode_cascade: batch tables too short");
  void* outp = nullptr;
  void* o8 = nullptr;
  void* mxp = nullptr;
  int mx_rows = 0;
  if (mxo) {
    CHECK_GPU(*out8); CHECK_CONTIG(*out8); CHECK_GPU(*mx); CHECK_CONTIG(*mx); CHECK_DTYPE(*mx, at::kByte);
    TORCH_CHECK(out8->scalar_type() == at::kFloat8_e4m3fn && out8->numel() >= (int64_t)B * Hq * D,
                "paged_decode_cascade: out8 must be e4m3 [B, Hq * D]");
    TORCH_CHECK(mx->dim() == 3 && mx->size(0) == Hq && mx->size(1) >= B && mx->size(2) == 4 && D == 128,
                "paged_decode_cascade: mx must be [Hq, B, 4] (head_dim 128)");
    o8 = out8->data_ptr();
    mxp = mx->data_ptr();
    mx_rows = (int)mx->size(1);
  } else {
    CHECK_BF16(*out); CHECK_CONTIG(*out);
    TORCH_CHECK(out->numel() >= (int64_t)B * Hq * D, "paged_decode_cascade: out too small");
    outp = out->data_ptr();
  }
  const QRope qr = q_rope(rope_cos, rope_sin, positions, B, D, "paged_decode_cascade");
  CHECK_RC(lwc_paged_decode_cascade(q.data_ptr(), (int)q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                                    block_tables.data_ptr<int>(), ctx_lens.data_ptr<int>(), tiles.data_ptr<int>(),
                                    (int)tiles.size(0), outp, (int)Hq, Hkv, D, BS,
                                    (int)block_tables.size(1), (float)scale, qr.cos, qr.sin, qr.pos, o8, mxp, mx_rows,
                                    cur_stream()),
           "paged_decode_cascade");
}

void grouped_gemm(const at::Tensor& A, const at::Tensor& W, at::Tensor& C, const at::Tensor& row_off, int64_t max_slots,
                  const c10::optional<at::Tensor>& a_scale, const c10::optional<at::Tensor>& w_scale,
                  const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& a_rows, int64_t splits) {
  // A [rows, K] (bf16 | fp8 e4m3fn, unit inner stride), W [G, N, K] contiguous, C [rows, N] bf16,
  // row_off [G+1] int32 on the device (group boundaries; the kernel trusts them to be <= rows).
  CHECK_GPU(A); CHECK_GPU(W); CHECK_BF16(C); CHECK_DTYPE(row_off, at::kInt); CHECK_CONTIG(row_off);
  CHECK_CONTIG(W);
  const bool fp8 = A.scalar_type() == at::kFloat8_e4m3fn;
  TORCH_CHECK(fp8 ? W.scalar_type() == at::kFloat8_e4m3fn : (A.scalar_type() == at::kBFloat16 &&
              W.scalar_type() == at::kBFloat16), "grouped_gemm: A/W must both be bf16 or both fp8 e4m3fn");
  TORCH_CHECK(A.dim() == 2 && A.stride(1) == 1 && C.dim() == 2 && C.stride(1) == 1, "grouped_gemm: 2-D row-major A/C");
  TORCH_CHECK(W.dim() == 3, "grouped_gemm: W must be [G, N, K]");
  const int G = (int)W.size(0), N = (int)W.size(1), K = (int)W.size(2);
  TORCH_CHECK(A.size(1) == K && C.size(1) == N, "grouped_gemm: shape mismatch");
  const int* ar = nullptr;
  if (a_rows.has_value() && a_rows->defined()) {
    CHECK_DTYPE(*a_rows, at::kInt); CHECK_CONTIG(*a_rows);
    TORCH_CHECK(a_rows->numel() >= C.size(0), "grouped_gemm: a_rows shorter than the output rows");
    ar = a_rows->data_ptr<int>();
  } else {
    TORCH_CHECK(C.size(0) >= A.size(0), "grouped_gemm: C rows < A rows");
  }
  TORCH_CHECK(row_off.numel() == G + 1, "grouped_gemm: row_off must have G+1 entries");
  const float* as = nullptr;
  const float* ws = nullptr;
  if (fp8) {
    TORCH_CHECK(a_scale.has_value() && w_scale.has_value(), "grouped_gemm: fp8 needs a_scale and w_scale");
    CHECK_DTYPE(*a_scale, at::kFloat); CHECK_DTYPE(*w_scale, at::kFloat);
    TORCH_CHECK(a_scale->numel() >= A.size(0) && w_scale->numel() == (int64_t)G * N, "grouped_gemm: scale shapes");
    as = a_scale->data_ptr<float>();
    ws = w_scale->data_ptr<float>();
  }
  const void* b = nullptr;
  if (bias.has_value() && bias->defined()) {
    CHECK_BF16(*bias);
    TORCH_CHECK(bias->numel() == (int64_t)G * N, "grouped_gemm: bias must be [G, N]");
    b = bias->data_ptr();
  }
  TORCH_CHECK(splits >= 1, "grouped_gemm: splits must be >= 1");
  at::Tensor c32;  // split-K: fp32 accumulation buffer over all output rows
  if (splits > 1) c32 = at::zeros({C.size(0), N}, C.options().dtype(at::kFloat));
  CHECK_RC(lwc_grouped_gemm(A.data_ptr(), W.data_ptr(), C.data_ptr(), row_off.data_ptr<int>(), as, ws, b, ar, G,
                            (int)max_slots, N, K, (int)A.stride(0), (int)C.stride(0), (long long)N * K, fp8 ? 1 : 0,
                            splits > 1 ? c32.data_ptr<float>() : nullptr, (int)splits, (long long)C.size(0),
                            cur_stream()),
           "grouped_gemm");
}

// Operand checks shared by the MFMA GEMM cores; returns the epilogue operand (residual / bias) or null.
const void* gemm_operands(const at::Tensor& A, const at::Tensor& W, const at::Tensor& C,
                          const c10::optional<at::Tensor>& R, int64_t epi) {
  // epi 0: C[M, N] = A . W^T; 1: + R; 2: C[M, N/2] = silu(gate) * up over a 32-row gate/up interleaved W;
  // 3: + bias (R = bias [N]); 4: gelu(. + bias)
  CHECK_BF16(A); CHECK_BF16(W); CHECK_BF16(C); CHECK_CONTIG(W);
  TORCH_CHECK(A.dim() == 2 && A.stride(1) == 1 && C.dim() == 2 && C.stride(1) == 1, "gemm8p: 2-D row-major A/C");
  TORCH_CHECK(epi >= 0 && epi <= 4, "gemm8p: epi must be 0..4");
  const int M = (int)A.size(0), K = (int)A.size(1), N = (int)W.size(0);
  const int NC = epi == 2 ? N / 2 : N;
  TORCH_CHECK(W.size(1) == K && C.size(0) == M && C.size(1) == NC, "gemm8p: shape mismatch");
  TORCH_CHECK(K % 64 == 0 && N % (epi == 2 ? 64 : 8) == 0 && A.stride(0) % 8 == 0 && C.stride(0) % 8 == 0,
              "gemm8p: needs K % 64 == 0, N % 8 == 0 (SwiGLU: N % 64 == 0) and 16-byte aligned rows");
  const void* r = nullptr;
  if (epi == 1) {
    TORCH_CHECK(R.has_value() && R->defined(), "gemm8p: epi 1 needs a residual");
    CHECK_BF16(*R);
    TORCH_CHECK(R->sizes() == C.sizes() && R->strides() == C.strides(), "gemm8p: residual must match C");
    r = R->data_ptr();
  }
  if (epi == 3 || epi == 4) {
    TORCH_CHECK(R.has_value() && R->defined(), "gemm8p: bias epilogue needs a bias");
    CHECK_BF16(*R); CHECK_CONTIG(*R);
    TORCH_CHECK(R->numel() == N, "gemm8p: bias must have N elements");
    r = R->data_ptr();
  }
  return r;
}

void gemm8p(const at::Tensor& A, const at::Tensor& W, at::Tensor& C, const c10::optional<at::Tensor>& R, int64_t epi,
            at::Tensor& ws, at::Tensor& flags) {
  const void* r = gemm_operands(A, W, C, R, epi);
  const int M = (int)A.size(0), K = (int)A.size(1), N = (int)W.size(0);
  // stream-K workspace: one fp32 256x256 partial tile and one flag per workgroup (flags zero between calls)
  const int slots = lwc_gemm8p_slots();
  CHECK_GPU(ws); CHECK_DTYPE(ws, at::kFloat); CHECK_CONTIG(ws);
  CHECK_GPU(flags); CHECK_DTYPE(flags, at::kInt); CHECK_CONTIG(flags);
  TORCH_CHECK(ws.numel() >= (int64_t)slots * 65536 && flags.numel() >= slots, "gemm8p: workspace too small (",
              slots, " slots)");
  CHECK_RC(lwc_gemm8p(A.data_ptr(), W.data_ptr(), C.data_ptr(), r, ws.data_ptr<float>(), flags.data_ptr<int>(), M, N,
                      K, (int)A.stride(0), (int)C.stride(0), (int)epi, cur_stream()),
           "gemm8p");
}

// gemm4w: the 4-wave interleaved core (one wave per SIMD, data-parallel tiles of 256 x bn, bn = 256 | 192).
// Folded RMSNorm (gemm4w.hip head): rs_mode 1 (epi 0 / 2) reads ss [>= P, M] fp32 partial row sums of squares
// and scales the accumulator rows by rsqrt(sum / K + eps); rs_mode 2 (epi 1, bn 256) writes ss [N/256, M].
void gemm4w(const at::Tensor& A, const at::Tensor& W, at::Tensor& C, const c10::optional<at::Tensor>& R, int64_t epi,
            int64_t bn, const c10::optional<at::Tensor>& ss, int64_t rs_mode, int64_t P, double eps, int64_t var,
            int64_t gm, int64_t splits, int64_t split_from, const c10::optional<at::Tensor>& part,
            const c10::optional<at::Tensor>& cnt) {
  const void* r = gemm_operands(A, W, C, R, epi);
  const int M = (int)A.size(0), K = (int)A.size(1), N = (int)W.size(0);
  TORCH_CHECK(bn == 256 || bn == 192, "gemm4w: bn must be 256 or 192");
  TORCH_CHECK(epi != 2 || bn == 256, "gemm4w: SwiGLU needs bn 256");
  float* ssp = nullptr;
  if (rs_mode) {
    TORCH_CHECK(ss.has_value() && ss->defined(), "gemm4w: rs_mode needs ss");
    CHECK_GPU(*ss); CHECK_DTYPE(*ss, at::kFloat); CHECK_CONTIG(*ss);
    TORCH_CHECK(ss->dim() == 2 && ss->size(1) >= M && ss->size(1) % 4 == 0, "gemm4w: ss [partials, >= M (x4)]");
    if (rs_mode == 1) {
      TORCH_CHECK(epi == 0 || epi == 2, "gemm4w: row scales go with the plain or SwiGLU epilogue");
      TORCH_CHECK(P >= 1 && P <= 16 && ss->size(0) >= P, "gemm4w: ss needs P (1..16) partials");
    } else {
      TORCH_CHECK(rs_mode == 2 && epi == 1 && bn == 256, "gemm4w: row sums of squares need the residual epilogue, bn 256");
      TORCH_CHECK(ss->size(0) >= (N + 255) / 256, "gemm4w: ss needs N/256 partials");
    }
    ssp = ss->data_ptr<float>();
  }
  if (splits > 1) {
    // split-K workspace, checked here against what the kernel will index (a short buffer would fault)
    const long long tiles = (long long)((M + 255) / 256) * ((N + bn - 1) / bn);
    const long long split_tiles = tiles - std::min<long long>(std::max<long long>(split_from, 0), tiles);
    TORCH_CHECK(part.has_value() && cnt.has_value(), "gemm4w: split-K needs part and cnt");
    CHECK_GPU(*part); CHECK_DTYPE(*part, at::kFloat); CHECK_CONTIG(*part);
    CHECK_GPU(*cnt); CHECK_DTYPE(*cnt, at::kInt); CHECK_CONTIG(*cnt);
    TORCH_CHECK(part->numel() >= split_tiles * (splits - 1) * 256 * bn, "gemm4w: split-K partial slab too small");
    TORCH_CHECK(cnt->numel() >= 2 * tiles, "gemm4w: split-K counters too small");
  }
  CHECK_RC(lwc_gemm4w(A.data_ptr(), W.data_ptr(), C.data_ptr(), r, M, N, K, (int)A.stride(0), (int)C.stride(0),
                      (int)epi, (int)bn, ssp, ssp ? (int)ss->size(1) : 0, (int)rs_mode, (int)P, (float)eps, (int)var,
                      (int)gm, (int)splits, (int)split_from,
                      part.has_value() ? part->data_ptr<float>() : nullptr,
                      cnt.has_value() ? cnt->data_ptr<int>() : nullptr, cur_stream()),
           "gemm4w");
}

// skinny GEMM (decode-sized M <= 64): C = A . W^T (epi 0), R + A . W^T (epi 1, R may be C) or the SwiGLU of
// a 32-row gate/up interleaved W (epi 2, C [M, N / 2])
void skinny_gemm(const at::Tensor& A, const at::Tensor& W, at::Tensor& C, const c10::optional<at::Tensor>& R,
                 int64_t epi) {
  TORCH_CHECK(epi >= 0 && epi <= 2, "skinny_gemm: epi 0 (plain), 1 (residual) or 2 (SwiGLU)");
  const void* r = gemm_operands(A, W, C, R, epi);
  const int M = (int)A.size(0), K = (int)A.size(1), N = (int)W.size(0);
  TORCH_CHECK(M <= 64 && K % 2048 == 0 && N % 16 == 0, "skinny_gemm: needs M <= 64, K % 2048 == 0, N % 16 == 0");
  CHECK_RC(lwc_skinny_gemm(A.data_ptr(), W.data_ptr(), C.data_ptr(), r, M, N, K, (int)A.stride(0), (int)C.stride(0),
                           (int)epi, cur_stream()),
           "skinny_gemm");
}

// ss[r] = sum(x[r]^2): the single partial of the folded RMSNorm for the first projection of a chain
void rms_rowsumsq(const at::Tensor& x, at::Tensor& ss) {
  CHECK_BF16(x); CHECK_CONTIG(x); CHECK_GPU(ss); CHECK_DTYPE(ss, at::kFloat); CHECK_CONTIG(ss);
  TORCH_CHECK(x.dim() == 2 && ss.numel() >= x.size(0), "rms_rowsumsq: x [M, d], ss [>= M]");
  CHECK_RC(lwc_rms_rowsumsq(x.data_ptr(), ss.data_ptr<float>(), (int)x.size(0), (int)x.size(1), cur_stream()),
           "rms_rowsumsq");
}

void gemm8g_fp8(const at::Tensor& A, const at::Tensor& W, at::Tensor& C, const c10::optional<at::Tensor>& row_off,
                int64_t max_slots, const c10::optional<at::Tensor>& a_rows, const c10::optional<at::Tensor>& a_scale,
                const at::Tensor& w_scale, int64_t mode, const c10::optional<at::Tensor>& a_mx,
                const c10::optional<at::Tensor>& mx_out) {
  // grouped fp8 GEMM on the 8-phase schedule (gemm8g.hip): A [rows_a, K] e4m3, W [G, N, K] e4m3, C [rows, N] bf16;
  // row_off None: the dense projection (G = 1, every output row).  mode 1: SwiGLU epilogue, C [rows, N / 2] bf16;
  // mode 2: SwiGLU epilogue with MX output, C [rows, N / 2] e4m3 + mx_out [N / 256, rows, 4] e8m0 (uint8);
  // a_mx [K / 128, rows_a, 4] e8m0: A's MX block scales (mode 0, no a_rows; a_scale unused)
  CHECK_GPU(A); CHECK_GPU(W); CHECK_CONTIG(W);
  TORCH_CHECK(mode >= 0 && mode <= 2, "gemm8g: mode 0, 1 or 2");
  TORCH_CHECK(A.scalar_type() == at::kFloat8_e4m3fn && W.scalar_type() == at::kFloat8_e4m3fn, "gemm8g: e4m3 A and W");
  TORCH_CHECK(A.dim() == 2 && A.stride(1) == 1 && C.dim() == 2 && C.stride(1) == 1 && W.dim() == 3, "gemm8g: layouts");
  if (mode == 2) {
    TORCH_CHECK(C.scalar_type() == at::kFloat8_e4m3fn, "gemm8g: MX output is e4m3");
  } else {
    CHECK_BF16(C);
  }
  const int G = (int)W.size(0), N = (int)W.size(1), K = (int)W.size(2);
  const int* ro = nullptr;
  if (row_off.has_value() && row_off->defined()) {
    CHECK_DTYPE(*row_off, at::kInt); CHECK_CONTIG(*row_off);
    TORCH_CHECK(row_off->numel() == G + 1, "gemm8g: row_off must have G + 1 entries");
    ro = row_off->data_ptr<int>();
  } else {
    TORCH_CHECK(G == 1, "gemm8g: dense mode (no row_off) takes one weight");
    TORCH_CHECK(max_slots >= (C.size(0) + 255) / 256, "gemm8g: dense mode needs ceil(rows / 256) slots");
  }
  TORCH_CHECK(A.size(1) == K && C.size(1) == (mode ? N / 2 : N), "gemm8g: shape mismatch");
  TORCH_CHECK(A.size(0) * A.stride(0) < (int64_t(1) << 31), "gemm8g: A spans >= 2 GiB (32-bit buffer range)");
  TORCH_CHECK(!mode || N % 64 == 0, "gemm8g: SwiGLU needs whole 64-row gate / up block pairs");
  CHECK_DTYPE(w_scale, at::kFloat); CHECK_CONTIG(w_scale);
  TORCH_CHECK(w_scale.numel() == (int64_t)G * N, "gemm8g: w_scale shape");
  const bool mxa = a_mx.has_value() && a_mx->defined();
  const float* as = nullptr;
  if (!mxa) {
    TORCH_CHECK(a_scale.has_value() && a_scale->defined(), "gemm8g: a_scale or a_mx required");
    CHECK_DTYPE(*a_scale, at::kFloat); CHECK_CONTIG(*a_scale);
    TORCH_CHECK(a_scale->numel() >= A.size(0), "gemm8g: a_scale shape");
    as = a_scale->data_ptr<float>();
  }
  const int* ar = nullptr;
  if (a_rows.has_value() && a_rows->defined()) {
    CHECK_DTYPE(*a_rows, at::kInt); CHECK_CONTIG(*a_rows);
    TORCH_CHECK(a_rows->numel() >= C.size(0), "gemm8g: a_rows shorter than the output rows");
    ar = a_rows->data_ptr<int>();
  } else {
    TORCH_CHECK(C.size(0) <= A.size(0), "gemm8g: more output rows than A rows");
  }
  // scale planes [K / 128][rows][4] bytes; a row-range view of a larger tensor is accepted (the plane stride
  // is then the full tensor's row count)
  auto plane_rows = [](const at::Tensor& t, const char* what) {
    CHECK_GPU(t); CHECK_DTYPE(t, at::kByte);
    TORCH_CHECK(t.dim() == 3 && t.size(2) == 4 && t.stride(2) == 1 && t.stride(1) == 4 && t.stride(0) % 4 == 0 &&
                    t.stride(0) / 4 >= t.size(1),
                what, ": MX scales must be [K / 128, rows, 4] bytes with rows contiguous");
    return (int)(t.stride(0) / 4);
  };
  int s_rows = 0;
  const void* amx = nullptr;
  void* mxo = nullptr;
  if (mxa) {
    TORCH_CHECK(mode == 0 && ar == nullptr, "gemm8g: MX A takes the plain epilogue and contiguous rows");
    s_rows = plane_rows(*a_mx, "gemm8g a_mx");
    TORCH_CHECK(a_mx->size(0) == K / 128 && a_mx->size(1) >= A.size(0), "gemm8g: a_mx must be [K / 128, rows_a, 4]");
    amx = a_mx->data_ptr();
  }
  if (mode == 2) {
    TORCH_CHECK(mx_out.has_value() && mx_out->defined(), "gemm8g: mode 2 writes mx_out");
    s_rows = plane_rows(*mx_out, "gemm8g mx_out");
    TORCH_CHECK(N % 256 == 0 && mx_out->size(0) == N / 256 && mx_out->size(1) >= C.size(0) && C.stride(0) % 16 == 0,
                "gemm8g: mx_out must be [N / 256, rows, 4] (N % 256 == 0)");
    mxo = mx_out->data_ptr();
  }
  CHECK_RC(lwc_gemm8g_fp8(A.data_ptr(), W.data_ptr(), C.data_ptr(), ro, ar, as, w_scale.data_ptr<float>(), G,
                          (int)max_slots, N, K, (int)A.stride(0), (int)C.stride(0), (int)A.size(0), (int)C.size(0),
                          (int)mode, amx, mxo, s_rows, cur_stream()),
           "gemm8g_fp8");
}

void moe_route(const at::Tensor& logits, int64_t k, at::Tensor& topk_ids, at::Tensor& topk_w, at::Tensor& row_off,
               at::Tensor& src_row, at::Tensor& inv) {
  CHECK_BF16(logits); CHECK_CONTIG(logits);
  TORCH_CHECK(logits.dim() == 2, "moe_route: logits must be [T, E]");
  const int T = (int)logits.size(0), E = (int)logits.size(1);
  for (const at::Tensor* t : {&topk_ids, &row_off, &src_row, &inv}) {
    CHECK_GPU(*t); CHECK_DTYPE(*t, at::kInt); CHECK_CONTIG(*t);
  }
  CHECK_DTYPE(topk_w, at::kFloat); CHECK_CONTIG(topk_w);
  TORCH_CHECK(topk_ids.numel() >= (int64_t)T * k && topk_w.numel() >= (int64_t)T * k && src_row.numel() >= (int64_t)T * k &&
              inv.numel() >= (int64_t)T * k && row_off.numel() == E + 1, "moe_route: output sizes");
  CHECK_RC(lwc_moe_route(logits.data_ptr(), T, E, (int)k, topk_ids.data_ptr<int>(), topk_w.data_ptr<float>(),
                         row_off.data_ptr<int>(), src_row.data_ptr<int>(), inv.data_ptr<int>(), cur_stream()),
           "moe_route");
}

void moe_router(const at::Tensor& h, const at::Tensor& router, int64_t k, at::Tensor& topk_ids, at::Tensor& topk_w,
                at::Tensor& row_off, at::Tensor& src_row, at::Tensor& inv, const c10::optional<at::Tensor>& logits) {
  CHECK_BF16(h); CHECK_BF16(router); CHECK_CONTIG(router);
  TORCH_CHECK(h.dim() == 2 && router.dim() == 2 && h.size(1) == router.size(1) && h.stride(1) == 1,
              "moe_router: h [T, d] (unit column stride), router [E, d]");
  const int T = (int)h.size(0), E = (int)router.size(0), d = (int)h.size(1);
  for (const at::Tensor* t : {&topk_ids, &row_off, &src_row, &inv}) {
    CHECK_GPU(*t); CHECK_DTYPE(*t, at::kInt); CHECK_CONTIG(*t);
  }
  CHECK_DTYPE(topk_w, at::kFloat); CHECK_CONTIG(topk_w);
  TORCH_CHECK(topk_ids.numel() >= (int64_t)T * k && topk_w.numel() >= (int64_t)T * k && src_row.numel() >= (int64_t)T * k &&
              inv.numel() >= (int64_t)T * k && row_off.numel() == E + 1, "moe_router: output sizes");
  if (logits.has_value()) {
    CHECK_BF16(*logits); CHECK_CONTIG(*logits);
    TORCH_CHECK(logits->numel() == (int64_t)T * E, "moe_router: logits [T, E]");
  }
  CHECK_RC(lwc_moe_router(h.data_ptr(), (int)h.stride(0), router.data_ptr(), T, E, d, (int)k, topk_ids.data_ptr<int>(),
                          topk_w.data_ptr<float>(), row_off.data_ptr<int>(), src_row.data_ptr<int>(),
                          inv.data_ptr<int>(), logits.has_value() ? logits->data_ptr() : nullptr, cur_stream()),
           "moe_router");
}

// C4 expert-parallel exchange buffers (csrc/kernels/ep.hip): send / recv are uint8 [W, (C + 1) * RB].
int64_t row_bytes_of(const at::Tensor& x) { return x.size(1) * (int64_t)x.element_size(); }

void ep_pack(const at::Tensor& x, const c10::optional<at::Tensor>& xs, const c10::optional<at::Tensor>& src,
             const at::Tensor& row_off, int64_t W, int64_t El, int64_t C, at::Tensor& send) {
  CHECK_GPU(x); CHECK_CONTIG(x); CHECK_GPU(send); CHECK_CONTIG(send); CHECK_DTYPE(send, at::kByte);
  CHECK_DTYPE(row_off, at::kInt);
  TORCH_CHECK(x.dim() == 2 && row_off.numel() == W * El + 1, "ep_pack: x [rows, d], row_off [W*El+1]");
  TORCH_CHECK(send.dim() == 2 && send.size(0) == W && send.size(1) % (C + 1) == 0, "ep_pack: send [W, (C+1)*RB]");
  if (src.has_value()) { CHECK_DTYPE(*src, at::kInt); CHECK_CONTIG(*src); }
  if (xs.has_value()) { CHECK_DTYPE(*xs, at::kFloat); TORCH_CHECK(xs->numel() == x.size(0), "ep_pack: one scale per row"); }
  CHECK_RC(lwc_ep_pack(x.data_ptr(), opt_ptr<float>(xs), opt_ptr<int>(src), row_off.data_ptr<int>(), (int)W, (int)El,
                       (int)C, (int)(send.size(1) / (C + 1)), (int)row_bytes_of(x), send.data_ptr(), cur_stream()),
           "ep_pack");
}

void ep_unpack(const at::Tensor& recv, int64_t W, int64_t El, int64_t C, at::Tensor& x_local,
               const c10::optional<at::Tensor>& s_local, at::Tensor& map, at::Tensor& row_off_local) {
  CHECK_GPU(recv); CHECK_CONTIG(recv); CHECK_DTYPE(recv, at::kByte); CHECK_CONTIG(x_local);
  CHECK_DTYPE(map, at::kInt); CHECK_DTYPE(row_off_local, at::kInt);
  TORCH_CHECK(recv.dim() == 2 && recv.size(0) == W && recv.size(1) % (C + 1) == 0, "ep_unpack: recv [W, (C+1)*RB]");
  TORCH_CHECK(x_local.dim() == 2 && x_local.size(0) == W * C && map.numel() == W * C && row_off_local.numel() == El + 1,
              "ep_unpack: x_local [W*C, d], map [W*C], row_off_local [El+1]");
  if (s_local.has_value()) {
    CHECK_DTYPE(*s_local, at::kFloat);
    TORCH_CHECK(s_local->numel() == W * C, "ep_unpack: s_local [W*C]");
  }
  CHECK_RC(lwc_ep_unpack(recv.data_ptr(), (int)W, (int)El, (int)C, (int)(recv.size(1) / (C + 1)),
                         (int)row_bytes_of(x_local), s_local.has_value() ? 1 : 0, x_local.data_ptr(),
                         s_local.has_value() ? s_local->data_ptr<float>() : nullptr, map.data_ptr<int>(),
                         row_off_local.data_ptr<int>(), cur_stream()),
           "ep_unpack");
}

void ep_back(const at::Tensor& y_local, const at::Tensor& map, int64_t W, int64_t C, at::Tensor& back) {
  CHECK_GPU(y_local); CHECK_CONTIG(y_local); CHECK_CONTIG(back); CHECK_DTYPE(map, at::kInt);
  TORCH_CHECK(y_local.dim() == 2 && y_local.size(0) >= W * C && back.dim() == 2 && back.size(0) == W * C &&
                  back.size(1) == y_local.size(1) && back.scalar_type() == y_local.scalar_type() && map.numel() == W * C,
              "ep_back: y_local [>= W*C, d], back [W*C, d], map [W*C]");
  CHECK_RC(lwc_ep_back(y_local.data_ptr(), map.data_ptr<int>(), (int)W, (int)C, (int)row_bytes_of(y_local),
                       back.data_ptr(), cur_stream()),
           "ep_back");
}

void ep_combine(const at::Tensor& ret, const at::Tensor& row_off, const at::Tensor& inv, const at::Tensor& w,
                int64_t El, int64_t C, int64_t k, at::Tensor& out) {
  CHECK_BF16(ret); CHECK_BF16(out); CHECK_CONTIG(ret); CHECK_CONTIG(out);
  CHECK_DTYPE(row_off, at::kInt); CHECK_DTYPE(inv, at::kInt); CHECK_DTYPE(w, at::kFloat);
  const int T = (int)out.size(0), d = (int)out.size(1);
  const int64_t E = row_off.numel() - 1;
  TORCH_CHECK(ret.size(1) == d && ret.size(0) == (E / El) * C && inv.numel() >= (int64_t)T * k &&
                  w.numel() >= (int64_t)T * k,
              "ep_combine: ret [W*C, d], inv / w [T*k]");
  CHECK_RC(lwc_ep_combine(ret.data_ptr(), row_off.data_ptr<int>(), inv.data_ptr<int>(), w.data_ptr<float>(), T, (int)E,
                          (int)El, (int)C, (int)k, d, out.data_ptr(), cur_stream()),
           "ep_combine");
}

void moe_combine(const at::Tensor& Y, const at::Tensor& inv, const at::Tensor& w, int64_t k, at::Tensor& out) {
  CHECK_BF16(Y); CHECK_BF16(out); CHECK_CONTIG(Y); CHECK_CONTIG(out);
  CHECK_DTYPE(inv, at::kInt); CHECK_DTYPE(w, at::kFloat);
  const int T = (int)out.size(0), d = (int)out.size(1);
  TORCH_CHECK(Y.size(1) == d && inv.numel() >= (int64_t)T * k && w.numel() >= (int64_t)T * k, "moe_combine: shapes");
  CHECK_RC(lwc_moe_combine(Y.data_ptr(), inv.data_ptr<int>(), w.data_ptr<float>(), T, (int)k, d, out.data_ptr(),
                           cur_stream()),
           "moe_combine");
}

void quant_fp8_rows(const at::Tensor& x, at::Tensor& q, at::Tensor& scale) {
  CHECK_BF16(x); CHECK_CONTIG(x); CHECK_CONTIG(q);
  TORCH_CHECK(q.scalar_type() == at::kFloat8_e4m3fn && q.numel() == x.numel(), "quant_fp8_rows: q must be e4m3fn like x");
  CHECK_DTYPE(scale, at::kFloat);
  const int d = (int)x.size(-1), rows = (int)(x.numel() / d);
  TORCH_CHECK(scale.numel() >= rows, "quant_fp8_rows: scale too short");
  CHECK_RC(lwc_quant_fp8_rows(x.data_ptr(), rows, d, q.data_ptr(), scale.data_ptr<float>(), cur_stream()),
           "quant_fp8_rows");
}

void silu_mul_quant_fp8(const at::Tensor& gu, at::Tensor& q, at::Tensor& scale, int64_t block) {
  // gu [rows, 2F] bf16 (gate | up, or interleaved in blocks) -> q [rows, F] e4m3fn, scale [rows] f32
  CHECK_BF16(gu); CHECK_CONTIG(gu); CHECK_CONTIG(q); CHECK_DTYPE(scale, at::kFloat);
  TORCH_CHECK(gu.dim() == 2 && q.dim() == 2 && q.scalar_type() == at::kFloat8_e4m3fn, "silu_mul_quant_fp8: 2-D");
  const int rows = (int)gu.size(0), F = (int)q.size(1);
  TORCH_CHECK(gu.size(1) == 2 * F && q.size(0) == rows && scale.numel() >= rows, "silu_mul_quant_fp8: shape mismatch");
  TORCH_CHECK(block == 0 || (block % 8 == 0 && F % block == 0), "silu_mul_quant_fp8: bad block");
  CHECK_RC(lwc_silu_mul_quant_fp8(gu.data_ptr(), rows, F, (int)block, q.data_ptr(), scale.data_ptr<float>(),
                                  cur_stream()),
           "silu_mul_quant_fp8");
}

void prefill_attention(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, at::Tensor& out,
                       const at::Tensor& cu_seqlens, int64_t max_seqlen, int64_t Hq, int64_t Hkv, int64_t D,
                       double scale, bool causal, const c10::optional<at::Tensor>& cu_seqlens_k) {
  // q/k/v: [T, *] 2-D views with unit inner stride (slices of the fused qkv row); out: [T, Hq*D].
  // cu_seqlens_k (optional): per-sequence key ranges in k/v, each at least as long as the sequence's query
  // range (the caller checks the lengths on the host; queries are the last rows of the key range).
  CHECK_BF16(q); CHECK_BF16(k); CHECK_BF16(v); CHECK_BF16(out);
  CHECK_DTYPE(cu_seqlens, at::kInt);
  const int* cuk = nullptr;
  if (cu_seqlens_k.has_value()) {
    CHECK_DTYPE((*cu_seqlens_k), at::kInt);
    TORCH_CHECK(cu_seqlens_k->numel() == cu_seqlens.numel(), "prefill_attention: cu_seqlens_k size mismatch");
    TORCH_CHECK(k.size(0) == v.size(0), "prefill_attention: k/v row mismatch");
    cuk = cu_seqlens_k->data_ptr<int>();
  }
  TORCH_CHECK(q.dim() == 2 && k.dim() == 2 && v.dim() == 2 && out.dim() == 2, "prefill_attention: 2-D views expected");
  TORCH_CHECK(q.stride(1) == 1 && k.stride(1) == 1 && v.stride(1) == 1 && out.stride(1) == 1,
              "prefill_attention: unit inner stride");
  TORCH_CHECK(q.size(1) == Hq * D && k.size(1) == Hkv * D && v.size(1) == Hkv * D && out.size(1) == Hq * D,
              "prefill_attention: head shape mismatch");
  const int nseq = (int)cu_seqlens.numel() - 1;
  CHECK_RC(lwc_prefill_attention(q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), cu_seqlens.data_ptr<int>(),
                                 cuk, nseq, (int)max_seqlen, (int)q.stride(0), (int)k.stride(0), (int)v.stride(0),
                                 (int)out.stride(0), (int)Hq, (int)Hkv, (int)D, (float)scale, causal ? 1 : 0,
                                 cur_stream()),
           "prefill_attention");
}

void prefill_attention_mx(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, at::Tensor& out8, at::Tensor& mx,
                          const at::Tensor& cu_seqlens, int64_t max_seqlen, int64_t Hq, int64_t Hkv, double scale,
                          bool causal) {
  // D = 128; out8 [T, Hq*128] e4m3 (uint8 view, 16-B aligned row stride), mx [Hq, >= T, 4] uint8 contiguous
  CHECK_BF16(q); CHECK_BF16(k); CHECK_BF16(v); CHECK_DTYPE(cu_seqlens, at::kInt);
  CHECK_GPU(out8); CHECK_GPU(mx); CHECK_CONTIG(mx);
  TORCH_CHECK(out8.element_size() == 1 && mx.element_size() == 1, "prefill_attention_mx: byte outputs");
  TORCH_CHECK(q.dim() == 2 && k.dim() == 2 && v.dim() == 2 && out8.dim() == 2, "prefill_attention_mx: 2-D views");
  TORCH_CHECK(q.stride(1) == 1 && k.stride(1) == 1 && v.stride(1) == 1 && out8.stride(1) == 1 && out8.stride(0) % 16 == 0,
              "prefill_attention_mx: unit inner stride, 16-B row stride of out8");
  TORCH_CHECK(q.size(1) == Hq * 128 && k.size(1) == Hkv * 128 && v.size(1) == Hkv * 128 && out8.size(1) == Hq * 128 &&
                  out8.size(0) == q.size(0),
              "prefill_attention_mx: head shape mismatch (head_dim 128)");
  TORCH_CHECK(mx.dim() == 3 && mx.size(0) == Hq && mx.size(1) >= q.size(0) && mx.size(2) == 4,
              "prefill_attention_mx: mx [Hq, >= T, 4]");
  const int nseq = (int)cu_seqlens.numel() - 1;
  CHECK_RC(lwc_prefill_attention_mx(q.data_ptr(), k.data_ptr(), v.data_ptr(), out8.data_ptr(), mx.data_ptr(),
                                    (int)mx.size(1), cu_seqlens.data_ptr<int>(), nseq, (int)max_seqlen,
                                    (int)q.stride(0), (int)k.stride(0), (int)v.stride(0), (int)out8.stride(0), (int)Hq,
                                    (int)Hkv, (float)scale, causal ? 1 : 0, cur_stream()),
           "prefill_attention_mx");
}

void prefill_attention_paged(const at::Tensor& q, const at::Tensor& k_cache, const at::Tensor& v_cache, at::Tensor& out,
                             const at::Tensor& cu_seqlens, const at::Tensor& block_tables, const at::Tensor& k_lens,
                             int64_t max_seqlen, int64_t Hq, double scale) {
  // q [T, >=Hq*D] (row stride allowed), out [T, Hq*D]; K [NB, Hkv, 16, 128], V [NB, Hkv, 4, 128, 4];
  // block_tables [nseq, W] int32 (W even and >= 2 * ceil(max k_len / 32): a 32-key tile reads 2 entries),
  // k_lens [nseq] int32 (>= each sequence's query count: the queries are the last positions).
  CHECK_BF16(q); CHECK_BF16(out); CHECK_BF16(k_cache); CHECK_BF16(v_cache);
  CHECK_DTYPE(cu_seqlens, at::kInt); CHECK_DTYPE(block_tables, at::kInt); CHECK_DTYPE(k_lens, at::kInt);
  CHECK_CONTIG(block_tables); CHECK_CONTIG(k_lens);
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(2) == 16 && k_cache.size(3) == 128 && k_cache.is_contiguous(),
              "prefill_attention_paged: K cache [NB, Hkv, 16, 128]");
  check_v_cache(v_cache, k_cache, "prefill_attention_paged");
  const int Hkv = (int)k_cache.size(1), D = 128;
  const int nseq = (int)cu_seqlens.numel() - 1;
  TORCH_CHECK(block_tables.dim() == 2 && block_tables.size(0) == nseq && block_tables.size(1) % 2 == 0 &&
                  k_lens.numel() == nseq,
              "prefill_attention_paged: block_tables [nseq, even W] and k_lens [nseq]");
  TORCH_CHECK(q.dim() == 2 && out.dim() == 2 && q.stride(1) == 1 && out.stride(1) == 1 && q.size(1) >= Hq * D &&
                  out.size(1) == Hq * D && Hq % Hkv == 0,
              "prefill_attention_paged: q / out shapes");
  CHECK_RC(lwc_prefill_attention_paged(q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), out.data_ptr(),
                                       cu_seqlens.data_ptr<int>(), block_tables.data_ptr<int>(), k_lens.data_ptr<int>(),
                                       (int)block_tables.size(1), nseq, (int)max_seqlen, (int)q.stride(0),
                                       (int)out.stride(0), (int)Hq, Hkv, D, (float)scale, cur_stream()),
           "prefill_attention_paged");
}

void sample(const at::Tensor& logits, const at::Tensor& temperature, const at::Tensor& top_p, const at::Tensor& top_k,
            const at::Tensor& min_p, const at::Tensor& top_a, const c10::optional<at::Tensor>& freq_pen,
            const c10::optional<at::Tensor>& pres_pen, const c10::optional<at::Tensor>& rep_pen,
            const c10::optional<at::Tensor>& counts, const c10::optional<at::Tensor>& count_rows,
            const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& bias_rows,
            const c10::optional<at::Tensor>& mask, const c10::optional<at::Tensor>& mask_rows,
            const at::Tensor& seeds, const at::Tensor& offsets, int64_t num_logprobs, at::Tensor& out_token,
            at::Tensor& out_logprob, at::Tensor& out_topk_ids, at::Tensor& out_topk_lp, bool mask_logprobs,
            bool need_logprob) {
  CHECK_BF16(logits);
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "sample: logits must be [B, V] with unit inner stride");
  const int B = (int)logits.size(0), V = (int)logits.size(1);
  for (const at::Tensor* t : {&temperature, &top_p, &min_p, &top_a}) {
    CHECK_DTYPE(*t, at::kFloat);
    TORCH_CHECK(t->numel() >= B, "sample: per-row parameter too short");
  }
  CHECK_DTYPE(top_k, at::kInt);
  CHECK_DTYPE(seeds, at::kLong); CHECK_DTYPE(offsets, at::kLong);
  TORCH_CHECK(out_token.numel() >= B && out_logprob.numel() >= B, "sample: outputs too short");
  if (num_logprobs > 0)
    TORCH_CHECK(out_topk_ids.numel() >= B * num_logprobs && out_topk_lp.numel() >= B * num_logprobs,
                "sample: top-k outputs too short");
  if (counts.has_value() && counts->defined()) {
    TORCH_CHECK(counts->scalar_type() == at::kShort && counts->size(-1) == V, "sample: counts must be int16 [*, V]");
  }
  if (bias.has_value() && bias->defined()) TORCH_CHECK(bias->size(-1) == V, "sample: bias rows must be [*, V]");
  if (mask.has_value() && mask->defined()) TORCH_CHECK(mask->size(-1) == V / 32, "sample: mask rows must be [*, V/32]");
  CHECK_RC(lwc_sample(logits.data_ptr(), (int)logits.stride(0), V, B, temperature.data_ptr<float>(),
                      top_p.data_ptr<float>(), top_k.data_ptr<int>(), min_p.data_ptr<float>(), top_a.data_ptr<float>(),
                      opt_ptr<float>(freq_pen), opt_ptr<float>(pres_pen), opt_ptr<float>(rep_pen),
                      counts.has_value() && counts->defined() ? counts->data_ptr() : nullptr, opt_ptr<int>(count_rows),
                      opt_ptr<float>(bias), opt_ptr<int>(bias_rows), opt_ptr<unsigned int>(mask),
                      opt_ptr<int>(mask_rows), reinterpret_cast<const unsigned long long*>(seeds.data_ptr()),
                      reinterpret_cast<const unsigned long long*>(offsets.data_ptr()), (int)num_logprobs,
                      mask_logprobs ? 1 : 0, need_logprob ? 1 : 0, out_token.data_ptr<int>(), out_logprob.data_ptr<float>(),
                      num_logprobs > 0 ? out_topk_ids.data_ptr<int>() : nullptr,
                      num_logprobs > 0 ? out_topk_lp.data_ptr<float>() : nullptr, cur_stream()),
           "sample");
}

void pool_l2norm(const at::Tensor& hidden, const at::Tensor& cu_seqlens, int64_t mode, at::Tensor& out_f32,
                 const c10::optional<at::Tensor>& out_bf16) {
  CHECK_BF16(hidden); CHECK_DTYPE(cu_seqlens, at::kInt); CHECK_DTYPE(out_f32, at::kFloat);
  TORCH_CHECK(hidden.dim() == 2 && hidden.stride(1) == 1, "pool_l2norm: hidden must be [T, d]");
  const int nseq = (int)cu_seqlens.numel() - 1, d = (int)hidden.size(1);
  TORCH_CHECK(out_f32.numel() == (int64_t)nseq * d, "pool_l2norm: out shape");
  void* ob = nullptr;
  if (out_bf16.has_value() && out_bf16->defined()) {
    CHECK_BF16(*out_bf16);
    TORCH_CHECK(out_bf16->numel() == (int64_t)nseq * d, "pool_l2norm: bf16 out shape");
    ob = out_bf16->data_ptr();
  }
  CHECK_RC(lwc_pool_l2norm(hidden.data_ptr(), (int)hidden.stride(0), cu_seqlens.data_ptr<int>(), nseq, d, (int)mode,
                           out_f32.data_ptr<float>(), ob, cur_stream()),
           "pool_l2norm");
}

std::vector<at::Tensor> knn_topk(const at::Tensor& E, const at::Tensor& q, int64_t k) {
  // E [n, d] f32 (contiguous rows), q [d] f32 -> (values [k] f32, rows [k] int32), best first, ties to the lower row
  CHECK_GPU(E); CHECK_GPU(q); CHECK_CONTIG(E); CHECK_CONTIG(q);
  CHECK_DTYPE(E, at::kFloat); CHECK_DTYPE(q, at::kFloat);
  TORCH_CHECK(E.dim() == 2 && q.numel() == E.size(1) && E.size(1) % 4 == 0, "knn_topk: E [n, d] (d % 4 == 0), q [d]");
  const int n = (int)E.size(0), d = (int)E.size(1);
  TORCH_CHECK(k >= 1 && k <= 64 && k <= n, "knn_topk: 1 <= k <= min(64, n)");
  const int slabs = (n + 255) / 256;
  auto opts = E.options();
  at::Tensor pv = at::empty({2 * (int64_t)slabs * k}, opts), vals = at::empty({k}, opts);
  at::Tensor pi = at::empty({2 * (int64_t)slabs * k}, opts.dtype(at::kInt)), rows = at::empty({k}, opts.dtype(at::kInt));
  CHECK_RC(lwc_knn_topk(E.data_ptr<float>(), n, d, q.data_ptr<float>(), (int)k, pv.data_ptr<float>(),
                        pi.data_ptr<int>(), vals.data_ptr<float>(), rows.data_ptr<int>(), cur_stream()),
           "knn_topk");
  return {vals, rows};
}

std::vector<at::Tensor> vote_tally(const at::Tensor& V, const at::Tensor& w, const at::Tensor& valid) {
  // V [R, L, C] f64, w [R, L] f64, valid [R, L] u8 -> (choice weight [R, C], confidence [R, C],
  // voter confidence [R, L]; NaN where !valid)
  CHECK_GPU(V); CHECK_GPU(w); CHECK_GPU(valid); CHECK_CONTIG(V); CHECK_CONTIG(w); CHECK_CONTIG(valid);
  CHECK_DTYPE(V, at::kDouble); CHECK_DTYPE(w, at::kDouble); CHECK_DTYPE(valid, at::kByte);
  TORCH_CHECK(V.dim() == 3 && w.dim() == 2 && valid.dim() == 2, "vote_tally: V [R, L, C], w / valid [R, L]");
  const int R = (int)V.size(0), L = (int)V.size(1), C = (int)V.size(2);
  TORCH_CHECK(w.size(0) == R && w.size(1) == L && valid.size(0) == R && valid.size(1) == L,
              "vote_tally: w / valid must be [R, L]");
  TORCH_CHECK(C >= 1 && C <= 1024, "vote_tally: 1 <= choices <= 1024");
  at::Tensor cw = at::empty({R, C}, V.options()), conf = at::empty({R, C}, V.options());
  at::Tensor vconf = at::empty({R, L}, V.options());
  CHECK_RC(lwc_vote_tally(V.data_ptr<double>(), w.data_ptr<double>(), valid.data_ptr<uint8_t>(), R, L, C,
                          cw.data_ptr<double>(), conf.data_ptr<double>(), vconf.data_ptr<double>(), cur_stream()),
           "vote_tally");
  return {cw, conf, vconf};
}

void cosine_consensus(const at::Tensor& E, at::Tensor& S, double inv_tau, at::Tensor& centrality, at::Tensor& weights,
                      at::Tensor& best) {
  // E: [R, n, d] bf16; S: [R, n_pad, n_pad] f32
  CHECK_BF16(E); CHECK_CONTIG(E);
  TORCH_CHECK(E.dim() == 3, "cosine_consensus: E must be [R, n, d]");
  const int R = (int)E.size(0), n = (int)E.size(1), d = (int)E.size(2);
  const int n_pad = (n + 15) / 16 * 16;
  TORCH_CHECK(S.scalar_type() == at::kFloat && S.numel() >= (int64_t)R * n_pad * n_pad, "cosine_consensus: S size");
  TORCH_CHECK(centrality.numel() >= (int64_t)R * n && weights.numel() >= (int64_t)R * n && best.numel() >= R,
              "cosine_consensus: outputs too small");
  CHECK_RC(lwc_cosine_consensus(E.data_ptr(), R, n, d, S.data_ptr<float>(), (float)inv_tau,
                                centrality.data_ptr<float>(), weights.data_ptr<float>(), best.data_ptr<int>(),
                                cur_stream()),
           "cosine_consensus");
}

}  // namespace

// ---- C3 custom all-reduce (allreduce.hip): IPC regions are raw device pointers held by Python as ints
std::tuple<int64_t, py::bytes> ar_alloc(int64_t bytes) {
  void* ptr = nullptr;
  std::string h((size_t)lwc_ar_handle_bytes(), '\0');
  const int rc = lwc_ar_alloc(bytes, &ptr, h.data());
  TORCH_CHECK(rc == 0, "ar_alloc: HIP error ", rc);
  return {reinterpret_cast<int64_t>(ptr), py::bytes(h)};
}

int64_t ar_open(const py::bytes& handle) {
  std::string h = handle;
  TORCH_CHECK((int)h.size() == lwc_ar_handle_bytes(), "ar_open: bad handle size");
  void* ptr = nullptr;
  const int rc = lwc_ar_open(h.data(), &ptr);
  TORCH_CHECK(rc == 0, "ar_open: hipIpcOpenMemHandle failed with ", rc);
  return reinterpret_cast<int64_t>(ptr);
}

void ar_close(int64_t ptr) { (void)lwc_ar_close(reinterpret_cast<void*>(ptr)); }
void ar_free(int64_t ptr) { (void)lwc_ar_free(reinterpret_cast<void*>(ptr)); }
int64_t ar_region_bytes(int64_t W, int64_t cap) { return lwc_ar_region_bytes((int)W, cap); }

void allreduce(const std::vector<int64_t>& bases, int64_t me, const at::Tensor& x, at::Tensor& out, int64_t cap,
               at::Tensor& err, int64_t blocks, int64_t spin_limit) {
  CHECK_BF16(x); CHECK_BF16(out); CHECK_CONTIG(x); CHECK_CONTIG(out);
  CHECK_DTYPE(err, at::kInt);
  TORCH_CHECK(x.numel() == out.numel(), "allreduce: x / out size mismatch");
  TORCH_CHECK(x.numel() % 8 == 0, "allreduce: numel must be a multiple of 8");
  std::vector<void*> b;
  for (int64_t v : bases) b.push_back(reinterpret_cast<void*>(v));
  CHECK_RC(lwc_allreduce(b.data(), (int)me, (int)b.size(), x.data_ptr(), out.data_ptr(), x.numel(), cap,
                         err.data_ptr<int>(), (int)blocks, (long long)spin_limit, cur_stream()),
           "allreduce");
}

void alltoall(const std::vector<int64_t>& bases, int64_t me, const at::Tensor& send, at::Tensor& recv, int64_t cap,
              at::Tensor& err, int64_t blocks, int64_t spin_limit) {
  // equal-split all-to-all of raw bytes: send / recv [W, chunk] uint8 (chunk % 16 == 0)
  CHECK_GPU(send); CHECK_GPU(recv); CHECK_CONTIG(send); CHECK_CONTIG(recv);
  CHECK_DTYPE(send, at::kByte); CHECK_DTYPE(recv, at::kByte); CHECK_DTYPE(err, at::kInt);
  const int64_t W = (int64_t)bases.size();
  TORCH_CHECK(send.dim() == 2 && send.size(0) == W && recv.sizes() == send.sizes(), "alltoall: send / recv [W, chunk]");
  TORCH_CHECK(send.size(1) % 16 == 0 && send.size(1) <= cap, "alltoall: chunk % 16 == 0 and chunk <= cap");
  std::vector<void*> b;
  for (int64_t v : bases) b.push_back(reinterpret_cast<void*>(v));
  CHECK_RC(lwc_alltoall(b.data(), (int)me, (int)W, send.data_ptr(), recv.data_ptr(), send.size(1), cap,
                        err.data_ptr<int>(), (int)blocks, (long long)spin_limit, cur_stream()),
           "alltoall");
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "gfx950 HIP kernels of llm_weighted_consensus_amd";
  m.def("rmsnorm", &rmsnorm);
  m.def("rmsnorm_quant_fp8", &rmsnorm_quant_fp8);
  m.def("layernorm", &layernorm);
  m.def("rope_kv_write", &rope_kv_write);
  m.def("silu_mul", &silu_mul);
  m.def("embedding", &embedding);
  m.def("kv_block_copy", &kv_block_copy);
  m.def("paged_decode", &paged_decode);
  m.def("grouped_gemm", &grouped_gemm);
  m.def("gemm8p", &gemm8p);
  m.def("gemm4w", &gemm4w);
  m.def("skinny_gemm", &skinny_gemm);
  m.def("rms_rowsumsq", &rms_rowsumsq);
  m.def("gemm8p_slots", &lwc_gemm8p_slots);
  m.def("moe_route", &moe_route);
  m.def("moe_router", &moe_router);
  m.def("moe_combine", &moe_combine);
  m.def("quant_fp8_rows", &quant_fp8_rows);
  m.def("paged_decode_cascade", &paged_decode_cascade);
  m.def("cascade_rows_per_tile", &lwc_cascade_rows_per_tile, "sequences per cascade super-tile for a GQA ratio G");
  m.def("set_decode_wave_min_items", &lwc_set_decode_wave_min_items,
        "B*Hkv*splits threshold of the wave-per-item decode kernel; returns the previous value");
  m.def("prefill_attention", &prefill_attention);
  m.def("prefill_attention_mx", &prefill_attention_mx);
  m.def("prefill_attention_paged", &prefill_attention_paged);
  m.def("silu_mul_quant_fp8", &silu_mul_quant_fp8);
  m.def("kv_gather", &kv_gather);
  m.def("sample", &sample);
  m.def("pool_l2norm", &pool_l2norm);
  m.def("cosine_consensus", &cosine_consensus);
  m.def("knn_topk", &knn_topk);
  m.def("vote_tally", &vote_tally);
  m.def("gemm8g_fp8", &gemm8g_fp8);
  m.def("ar_alloc", &ar_alloc);
  m.def("ar_open", &ar_open);
  m.def("ar_close", &ar_close);
  m.def("ar_free", &ar_free);
  m.def("ar_region_bytes", &ar_region_bytes);
  m.def("allreduce", &allreduce);
  m.def("alltoall", &alltoall);
  m.def("ep_pack", &ep_pack);
  m.def("ep_unpack", &ep_unpack);
  m.def("ep_back", &ep_back);
  m.def("ep_combine", &ep_combine);
}
