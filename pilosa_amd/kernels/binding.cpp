// torch extension binding for the gfx950 bitmap kernels (module
// pilosa_amd._hipkernels).  Every entry point launches on torch's current HIP
// stream of the tensors' device, so the executor can overlap queries on
// separate streams and capture launch sequences in HIP graphs.
#include <ATen/hip/HIPContext.h>
#include <torch/extension.h>

#include <pybind11/numpy.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include "kernels.h"

namespace {

void check_dev(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a device tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

hipStream_t cur_stream(const torch::Tensor& t) {
  return at::hip::getCurrentHIPStream(t.device().index()).stream();
}

// Launch-time errors (bad grid, missing code object, ...) surface here
// instead of as a later, unrelated failure.
void check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  TORCH_CHECK(e == hipSuccess, what, ": kernel launch failed: ", hipGetErrorString(e));
}

// Small host int32 arrays (a batch's parameters) -> a new device tensor on
// the current stream, staged through a ring of pinned slots: one memcpy and
// one async H2D, no allocator or Python on the way.  A slot is rewritten only
// once the event recorded behind its previous copy has fired.
torch::Tensor upload_raw(const int32_t* src, int64_t n, int64_t device) {
  constexpr int NSLOT = 64;
  constexpr size_t SLOT_BYTES = 16384;
  static std::mutex mu;
  static char* ring = nullptr;
  static hipEvent_t ev[NSLOT];
  static bool used[NSLOT];
  static int next = 0;
  const size_t nb = size_t(n) * 4;
  auto out = torch::empty({n}, torch::TensorOptions().dtype(torch::kInt32).device(torch::kCUDA, device));
  if (nb == 0) return out;
  const hipStream_t st = at::hip::getCurrentHIPStream(int(device)).stream();
  if (nb > SLOT_BYTES) {   // large: pageable copy (rare)
    TORCH_CHECK(hipMemcpyAsync(out.data_ptr(), src, nb, hipMemcpyHostToDevice, st) == hipSuccess,
                "upload_i32 copy");
    // the source may be freed on return: this copy must have read it
    TORCH_CHECK(hipStreamSynchronize(st) == hipSuccess, "upload_i32 copy wait");
    return out;
  }
  std::lock_guard<std::mutex> g(mu);
  if (ring == nullptr) {
    TORCH_CHECK(hipHostMalloc(reinterpret_cast<void**>(&ring), NSLOT * SLOT_BYTES, hipHostMallocDefault) ==
                    hipSuccess, "upload_i32 pinned ring");
    for (int i = 0; i < NSLOT; i++) {
      TORCH_CHECK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) == hipSuccess, "upload_i32 event");
      used[i] = false;
    }
  }
  const int k = next;
  next = (next + 1) % NSLOT;
  if (used[k]) TORCH_CHECK(hipEventSynchronize(ev[k]) == hipSuccess, "upload_i32 slot wait");
  char* slot = ring + size_t(k) * SLOT_BYTES;
  std::memcpy(slot, src, nb);
  TORCH_CHECK(hipMemcpyAsync(out.data_ptr(), slot, nb, hipMemcpyHostToDevice, st) == hipSuccess, "upload_i32 copy");
  TORCH_CHECK(hipEventRecord(ev[k], st) == hipSuccess, "upload_i32 record");
  used[k] = true;
  return out;
}

torch::Tensor upload_i32(torch::Tensor host, int64_t device) {
  TORCH_CHECK(!host.is_cuda() && host.scalar_type() == torch::kInt32 && host.is_contiguous(), "host int32[]");
  return upload_raw(host.data_ptr<int32_t>(), host.numel(), device);
}

// Cache-only TopN batch parameters (topn_kernels.hip topn_cache_*):
// [lim Q | threshold Q | threshold index Q | keep Q | distinct thresholds T],
// n = 0 meaning every cached row (lim K, keep KK); n and thresholds clamped to
// int32, thresholds at least 1.  KK = the answer width.
struct TopNParams {
  std::vector<int32_t> prm;
  int64_t Q = 0, T = 0, KK = 0, maxlim = 0;
};

TopNParams pack_topn_params(const std::vector<int64_t>& ns, const std::vector<int64_t>& ths, int64_t K, int64_t U) {
  TopNParams p;
  const int64_t Q = int64_t(ns.size());
  TORCH_CHECK(Q > 0 && Q < 65536 && int64_t(ths.size()) == Q, "TopN batch: ns / thresholds");
  std::vector<int32_t> th(Q), uniq;
  bool all_n = true;
  int64_t nmx = 0;
  for (int64_t q = 0; q < Q; q++) {
    th[q] = int32_t(std::max<int64_t>(1, std::min<int64_t>(ths[q], INT32_MAX)));
    const int64_t n = std::max<int64_t>(0, std::min<int64_t>(ns[q], INT32_MAX));
    all_n = all_n && n != 0;
    nmx = std::max(nmx, n);
  }
  uniq = th;
  std::sort(uniq.begin(), uniq.end());
  uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
  p.Q = Q;
  p.T = int64_t(uniq.size());
  p.KK = all_n ? std::min(U, nmx) : U;
  p.prm.resize(4 * Q + p.T);
  int32_t* prm = p.prm.data();
  for (int64_t q = 0; q < Q; q++) {
    const int64_t n = std::max<int64_t>(0, std::min<int64_t>(ns[q], INT32_MAX));
    prm[q] = int32_t(n ? n : K);
    p.maxlim = std::max<int64_t>(p.maxlim, prm[q]);
    prm[Q + q] = th[q];
    prm[2 * Q + q] = int32_t(std::lower_bound(uniq.begin(), uniq.end(), th[q]) - uniq.begin());
    prm[3 * Q + q] = int32_t(n ? n : p.KK);
  }
  std::copy(uniq.begin(), uniq.end(), prm + 4 * Q);
  return p;
}

// Composite keys (count << 32 | ~index) of every query's kept answers in the
// host copy h[Q, KK + 1] (column 0 = the number kept) -> (ids uint64[],
// counts int64[], offsets[Q + 1]) with ids = space[index], or None when some
// query overflowed the select (column 0 < 0 or > KK).
py::object decode_topn_keys(const int64_t* h, int64_t Q, int64_t KK, const uint64_t* space, int64_t R) {
  std::vector<int64_t> offs(Q + 1, 0);
  for (int64_t q = 0; q < Q; q++) {
    const int64_t n = h[q * (KK + 1)];
    if (n < 0 || n > KK) return py::none();
    offs[q + 1] = offs[q] + n;
  }
  const int64_t total = offs[Q];
  py::array_t<uint64_t> ids(total);
  py::array_t<int64_t> cnts(total);
  uint64_t* pi = ids.mutable_data();
  int64_t* pc = cnts.mutable_data();
  for (int64_t q = 0; q < Q; q++) {
    const int64_t* k = h + q * (KK + 1) + 1;
    for (int64_t i = 0, n = offs[q + 1] - offs[q]; i < n; i++) {
      const int64_t d = int64_t(0xFFFFFFFFll) - (k[i] & 0xFFFFFFFFll);
      TORCH_CHECK(d >= 0 && d < R, "TopN answer: candidate ", d, " outside the ", R, " known rows");
      pi[offs[q] + i] = space[d];
      pc[offs[q] + i] = k[i] >> 32;
    }
  }
  return py::make_tuple(ids, cnts, offs);
}

void expr_count(torch::Tensor progs, torch::Tensor views, int64_t S, torch::Tensor out,
                c10::optional<torch::Tensor> per_key, int64_t mode, c10::optional<torch::Tensor> per_shard) {
  check_dev(progs, "progs");
  check_dev(views, "views");
  TORCH_CHECK(progs.numel() % sizeof(pk::QueryProg) == 0, "progs size");
  TORCH_CHECK(views.numel() % sizeof(pk::ViewDev) == 0, "views size");
  const int Q = int(progs.numel() / sizeof(pk::QueryProg));
  unsigned long long* o = nullptr;
  if (out.numel()) {
    check_dev(out, "out");
    TORCH_CHECK(out.scalar_type() == torch::kInt64 && out.numel() >= Q, "out must be int64[Q]");
    o = reinterpret_cast<unsigned long long*>(out.data_ptr<int64_t>());
  }
  int32_t* pk_ = nullptr;
  if (per_key.has_value() && per_key->numel()) {
    check_dev(*per_key, "per_key");
    TORCH_CHECK(per_key->scalar_type() == torch::kInt32 && per_key->numel() >= int64_t(Q) * S * 16,
                "per_key must be int32[Q*S*16]");
    pk_ = per_key->data_ptr<int32_t>();
  }
  int64_t* ps = nullptr;
  if (per_shard.has_value() && per_shard->numel()) {
    check_dev(*per_shard, "per_shard");
    TORCH_CHECK(per_shard->scalar_type() == torch::kInt64 && per_shard->numel() >= int64_t(Q) * S,
                "per_shard must be int64[Q*S]");
    ps = per_shard->data_ptr<int64_t>();
  }
  pk::launch_expr_count(reinterpret_cast<const pk::QueryProg*>(progs.data_ptr<uint8_t>()), Q,
                        reinterpret_cast<const pk::ViewDev*>(views.data_ptr<uint8_t>()), int(S), o, pk_, ps, int(mode),
                        cur_stream(progs));
  check_launch("expr_count");
}

void expr_materialize(torch::Tensor progs, torch::Tensor views, int64_t S, torch::Tensor counts,
                      torch::Tensor offs, torch::Tensor outp) {
  check_dev(progs, "progs");
  check_dev(views, "views");
  check_dev(counts, "counts");
  check_dev(offs, "offs");
  check_dev(outp, "outp");
  const int Q = int(progs.numel() / sizeof(pk::QueryProg));
  TORCH_CHECK(counts.numel() >= int64_t(Q) * S * 16 && offs.numel() >= int64_t(Q) * S * 16, "counts/offs size");
  pk::launch_expr_materialize(reinterpret_cast<const pk::QueryProg*>(progs.data_ptr<uint8_t>()), Q,
                              reinterpret_cast<const pk::ViewDev*>(views.data_ptr<uint8_t>()), int(S),
                              counts.data_ptr<int32_t>(), offs.data_ptr<int64_t>(),
                              reinterpret_cast<uint16_t*>(outp.data_ptr<int16_t>()), cur_stream(progs));
  check_launch("expr_materialize");
}

pk::BsiArgs bsi_args_from(const torch::Tensor& bsi_args) {
  TORCH_CHECK(!bsi_args.is_cuda() && bsi_args.scalar_type() == torch::kInt64 && bsi_args.numel() == 67,
              "bsi_args must be a cpu int64[67]: view, depth, exists, sign, bit_row[63]");
  auto a = bsi_args.data_ptr<int64_t>();
  pk::BsiArgs b{};
  b.view = int32_t(a[0]);
  b.depth = int32_t(a[1]);
  TORCH_CHECK(b.depth >= 0 && b.depth <= 63, "bsi depth");
  b.row_exists = a[2];
  b.row_sign = a[3];
  for (int i = 0; i < 64; i++) b.bit_row[i] = i < 63 ? a[4 + i] : -1;
  return b;
}

void bsi_range(torch::Tensor views, int64_t S, torch::Tensor bsi_args, int64_t op, int64_t p1, int64_t p2,
               torch::Tensor out_payload, torch::Tensor out_meta) {
  check_dev(views, "views");
  check_dev(out_payload, "out_payload");
  check_dev(out_meta, "out_meta");
  TORCH_CHECK(op >= 0 && op <= 7, "bsi op");
  TORCH_CHECK(out_payload.numel() >= S * 16 * 4096 && out_meta.numel() >= S * 16, "bsi_range outputs too small");
  TORCH_CHECK(out_meta.scalar_type() == torch::kInt64, "out_meta must be int64");
  pk::launch_bsi_range(reinterpret_cast<const pk::ViewDev*>(views.data_ptr<uint8_t>()), int(S), bsi_args_from(bsi_args),
                       int(op), p1, p2, reinterpret_cast<uint16_t*>(out_payload.data_ptr<int16_t>()),
                       out_meta.data_ptr<int64_t>(), nullptr, cur_stream(views));
  check_launch("bsi_range");
}

void bsi_range_count(torch::Tensor views, int64_t S, torch::Tensor bsi_args, int64_t op, int64_t p1, int64_t p2,
                     torch::Tensor out_count) {
  check_dev(views, "views");
  check_dev(out_count, "out_count");
  TORCH_CHECK(op >= 0 && op <= 7, "bsi op");
  TORCH_CHECK(out_count.scalar_type() == torch::kInt64 && out_count.numel() >= 1, "out_count int64[1]");
  pk::launch_bsi_range(reinterpret_cast<const pk::ViewDev*>(views.data_ptr<uint8_t>()), int(S), bsi_args_from(bsi_args),
                       int(op), p1, p2, nullptr, nullptr,
                       reinterpret_cast<unsigned long long*>(out_count.data_ptr<int64_t>()), cur_stream(views));
  check_launch("bsi_range_count");
}

void bsi_minmax(torch::Tensor progs, torch::Tensor views, int64_t S, torch::Tensor bsi_args, torch::Tensor out,
                int64_t which) {
  check_dev(progs, "progs");
  check_dev(views, "views");
  check_dev(out, "out");
  TORCH_CHECK(progs.numel() >= int64_t(sizeof(pk::QueryProg)), "one filter program required");
  TORCH_CHECK(out.scalar_type() == torch::kInt64 && out.numel() >= S * 16 * 10, "out must be int64[S*16*10]");
  pk::launch_bsi_minmax(reinterpret_cast<const pk::QueryProg*>(progs.data_ptr<uint8_t>()),
                        reinterpret_cast<const pk::ViewDev*>(views.data_ptr<uint8_t>()), int(S),
                        bsi_args_from(bsi_args), out.data_ptr<int64_t>(), cur_stream(views), int(which));
  check_launch("bsi_minmax");
}

void bsi_minmax_fold(torch::Tensor o, int64_t F, int64_t G, int64_t is_min, torch::Tensor out) {
  check_dev(o, "o");
  check_dev(out, "out");
  TORCH_CHECK(o.scalar_type() == torch::kInt64 && o.is_contiguous() && o.numel() == F * G * 10 && G > 0,
              "o must be int64[F*G*10]");
  TORCH_CHECK(F < (int64_t(1) << 31) - 1, "bsi_minmax_fold: fragment count");
  TORCH_CHECK(out.scalar_type() == torch::kInt64 && out.numel() >= 3, "out must be int64[3]");
  torch::Tensor part = torch::empty({((F + 63) / 64) * 4}, o.options());
  pk::launch_bsi_minmax_fold(o.data_ptr<int64_t>(), int(F), int(G), int(is_min), out.data_ptr<int64_t>(),
                             part.data_ptr<int64_t>(), cur_stream(o));
  check_launch("bsi_minmax_fold");
}

void bsi_sum(torch::Tensor progs, torch::Tensor views, int64_t S, torch::Tensor bsi_args, torch::Tensor out_sum,
             torch::Tensor out_cnt, int64_t fmode) {
  check_dev(progs, "progs");
  check_dev(views, "views");
  check_dev(out_sum, "out_sum");
  check_dev(out_cnt, "out_cnt");
  TORCH_CHECK(!bsi_args.is_cuda() && bsi_args.scalar_type() == torch::kInt64 && bsi_args.numel() == 67,
              "bsi_args must be a cpu int64[67]: view, depth, exists, sign, bit_row[63]");
  auto a = bsi_args.data_ptr<int64_t>();
  pk::BsiArgs b{};
  b.view = int32_t(a[0]);
  b.depth = int32_t(a[1]);
  TORCH_CHECK(b.depth >= 0 && b.depth <= 63, "bsi depth");
  b.row_exists = a[2];
  b.row_sign = a[3];
  for (int i = 0; i < 64; i++) b.bit_row[i] = i < 63 ? a[4 + i] : -1;
  const int Q = int(progs.numel() / sizeof(pk::QueryProg));
  pk::launch_bsi_sum(reinterpret_cast<const pk::QueryProg*>(progs.data_ptr<uint8_t>()), Q,
                     reinterpret_cast<const pk::ViewDev*>(views.data_ptr<uint8_t>()), int(S), b,
                     reinterpret_cast<unsigned long long*>(out_sum.data_ptr<int64_t>()),
                     reinterpret_cast<unsigned long long*>(out_cnt.data_ptr<int64_t>()), int(fmode),
                     cur_stream(progs));
  check_launch("bsi_sum");
}

void and2_count(torch::Tensor progs, torch::Tensor views, int64_t S, torch::Tensor pairs, torch::Tensor partial,
                int64_t cq, int64_t variant) {
  check_dev(progs, "progs");
  check_dev(views, "views");
  check_dev(pairs, "pairs");
  check_dev(partial, "partial");
  const int Q = int(progs.numel() / sizeof(pk::QueryProg));
  const int64_t n = int64_t(Q) * S * 16;
  TORCH_CHECK(pairs.numel() * pairs.element_size() >= n * 8, "pairs scratch must hold S*16*Q uint2");
  TORCH_CHECK(partial.scalar_type() == torch::kInt32 && partial.numel() >= n, "partial must be int32[S*16*Q]");
  pk::launch_and2_pairs(reinterpret_cast<const pk::QueryProg*>(progs.data_ptr<uint8_t>()), Q,
                        reinterpret_cast<const pk::ViewDev*>(views.data_ptr<uint8_t>()), int(S),
                        reinterpret_cast<uint2*>(pairs.data_ptr()), partial.data_ptr<int32_t>(), int(cq),
                        int(variant), cur_stream(progs));
  check_launch("and2_pairs");
}

pk::ViewDev viewdev_from(const torch::Tensor& vd);

#ifdef PK_KBENCH
void shadow_build(torch::Tensor view, int64_t S, torch::Tensor rows, torch::Tensor shadow) {
  check_dev(rows, "rows");
  check_dev(shadow, "shadow");
  TORCH_CHECK(rows.scalar_type() == torch::kInt32, "rows must be int32[R]");
  const int64_t R = rows.numel();
  TORCH_CHECK(shadow.scalar_type() == torch::kInt64 && shadow.is_contiguous() && shadow.numel() == R * S * 16 * 1024,
              "shadow must be int64[R*S*16*1024]");
  pk::ViewDev v = viewdev_from(view);
  TORCH_CHECK(R >= 0 && R < (int64_t(1) << 20) && S > 0, "shadow_build sizes");
  pk::launch_shadow_build(v, int(S), rows.data_ptr<int32_t>(), int(R), reinterpret_cast<uint64_t*>(shadow.data_ptr<int64_t>()),
                          cur_stream(shadow));
  check_launch("shadow_build");
}
#endif  // PK_KBENCH

void partial_sum_scatter(torch::Tensor partial, int64_t U, int64_t n, torch::Tensor ti, torch::Tensor out) {
  check_dev(partial, "partial");
  check_dev(ti, "ti");
  check_dev(out, "out");
  TORCH_CHECK(partial.scalar_type() == torch::kInt32 && partial.is_contiguous() && partial.numel() >= U * n,
              "partial must be int32[U*n]");
  TORCH_CHECK(ti.scalar_type() == torch::kInt64 && ti.numel() == n, "ti must be int64[n]");
  TORCH_CHECK(out.scalar_type() == torch::kInt64, "out must be int64");
  TORCH_CHECK(n < (int64_t(1) << 31) && U < (int64_t(1) << 40), "partial_sum_scatter sizes");
  // scatter indexes outside out are dropped in the kernel
  pk::launch_partial_sum_scatter(partial.data_ptr<int32_t>(), U, int(n), ti.data_ptr<int64_t>(),
                                 out.data_ptr<int64_t>(), out.numel(), cur_stream(partial));
  check_launch("partial_sum_scatter");
}

pk::ViewDev viewdev_from(const torch::Tensor& vd) {
  TORCH_CHECK(!vd.is_cuda() && vd.numel() * vd.element_size() == int64_t(sizeof(pk::ViewDev)),
              "view must be a cpu tensor holding one ViewDev (64 bytes)");
  pk::ViewDev v;
  memcpy(&v, vd.data_ptr(), sizeof(v));
  return v;
}

void topn_index(torch::Tensor view, int64_t S, int64_t K, int64_t k0, torch::Tensor cache_dense, torch::Tensor colcnt,
                torch::Tensor colptr, torch::Tensor entbase, torch::Tensor slots, bool fill) {
  check_dev(cache_dense, "cache_dense");
  check_dev(colcnt, "colcnt");
  TORCH_CHECK(cache_dense.scalar_type() == torch::kInt32 && cache_dense.numel() == S * K, "cache_dense int32[S*K]");
  TORCH_CHECK(colcnt.scalar_type() == torch::kInt32 && colcnt.numel() == S * (int64_t(1) << 20),
              "colcnt int32[S*2^20]");
  TORCH_CHECK(K > 0 && K <= 65535, "slot index needs 0 < K <= 65535");
  TORCH_CHECK(k0 >= 0 && k0 <= K, "slot index tail start 0 <= k0 <= K");
  const uint32_t* cp = nullptr;
  const int64_t* eb = nullptr;
  uint16_t* sl = nullptr;
  if (fill) {
    check_dev(colptr, "colptr");
    check_dev(entbase, "entbase");
    check_dev(slots, "slots");
    TORCH_CHECK(colptr.scalar_type() == torch::kInt32 && colptr.numel() == S * ((int64_t(1) << 20) + 1),
                "colptr int32[S*(2^20+1)]");
    TORCH_CHECK(entbase.scalar_type() == torch::kInt64 && entbase.numel() >= S, "entbase int64[S]");
    TORCH_CHECK(slots.scalar_type() == torch::kInt16, "slots int16");
    cp = reinterpret_cast<const uint32_t*>(colptr.data_ptr<int32_t>());
    eb = entbase.data_ptr<int64_t>();
    sl = reinterpret_cast<uint16_t*>(slots.data_ptr<int16_t>());
  }
  pk::launch_topn_index(viewdev_from(view), int(S), int(K), int(k0), cache_dense.data_ptr<int32_t>(),
                        reinterpret_cast<uint32_t*>(colcnt.data_ptr<int32_t>()), cp, eb, sl, fill,
                        cur_stream(cache_dense));
  check_launch("topn_index");
}

void leaf_src(torch::Tensor view, torch::Tensor rows, int64_t S, torch::Tensor counts, torch::Tensor offs,
              torch::Tensor has_run) {
  for (auto* t : {&rows, &counts, &offs, &has_run}) check_dev(*t, "leaf_src");
  const int64_t Q = rows.numel();
  TORCH_CHECK(rows.scalar_type() == torch::kInt64, "rows int64[Q]");
  TORCH_CHECK(counts.scalar_type() == torch::kInt32 && counts.numel() == Q * S * 16, "counts int32[Q*S*16]");
  TORCH_CHECK(offs.scalar_type() == torch::kInt64 && offs.numel() == Q * S * 16, "offs int64[Q*S*16]");
  TORCH_CHECK(has_run.scalar_type() == torch::kInt32 && has_run.numel() == 1, "has_run int32[1]");
  pk::launch_leaf_src(viewdev_from(view), rows.data_ptr<int64_t>(), int(Q), int(S), counts.data_ptr<int32_t>(),
                      offs.data_ptr<int64_t>(), has_run.data_ptr<int32_t>(), cur_stream(rows));
  check_launch("leaf_src");
}

void row_counts(torch::Tensor view, torch::Tensor shard_of, torch::Tensor dense, torch::Tensor out) {
  for (auto* t : {&shard_of, &dense, &out}) check_dev(*t, "row_counts");
  const int64_t N = dense.numel();
  TORCH_CHECK(shard_of.scalar_type() == torch::kInt32 && shard_of.numel() == N, "shard_of int32[N]");
  TORCH_CHECK(dense.scalar_type() == torch::kInt32, "dense int32[N]");
  TORCH_CHECK(out.scalar_type() == torch::kInt32 && out.numel() == N, "out int32[N]");
  pk::launch_row_counts(viewdev_from(view), shard_of.data_ptr<int32_t>(), dense.data_ptr<int32_t>(), N,
                        out.data_ptr<int32_t>(), cur_stream(dense));
  check_launch("row_counts");
}

void topn_cache_counts(torch::Tensor view, int64_t S, torch::Tensor u, torch::Tensor cm) {
  for (auto* t : {&u, &cm}) check_dev(*t, "topn_cache_counts");
  const int64_t U = u.numel();
  TORCH_CHECK(u.scalar_type() == torch::kInt32, "u int32[U]");
  TORCH_CHECK(cm.scalar_type() == torch::kInt32 && cm.numel() == U * S, "cm int32[U, S]");
  pk::launch_topn_cache_counts(viewdev_from(view), int(S), u.data_ptr<int32_t>(), int(U), cm.data_ptr<int32_t>(),
                               cur_stream(u));
  check_launch("topn_cache_counts");
}

void topn_cache_batch(torch::Tensor cnt, int64_t nmax, torch::Tensor inv, torch::Tensor u, torch::Tensor cm,
                      torch::Tensor prm, int64_t Q, int64_t T, torch::Tensor member, torch::Tensor tot,
                      torch::Tensor out, int64_t nlim) {
  TORCH_CHECK(nlim >= 0 && nlim <= nmax, "nlim: 0 (= nmax) .. nmax");
  for (auto* t : {&cnt, &inv, &u, &cm, &prm, &member, &tot, &out}) check_dev(*t, "topn_cache_batch");
  TORCH_CHECK(cnt.scalar_type() == torch::kInt32 && cnt.dim() == 2, "cnt int32[S, K]");
  const int64_t S = cnt.size(0), K = cnt.size(1), U = u.numel();
  TORCH_CHECK(nmax >= 0 && nmax <= K, "nmax out of range");
  TORCH_CHECK(inv.scalar_type() == torch::kInt32 && inv.numel() == S * nmax, "inv int32[S * nmax]");
  TORCH_CHECK(u.scalar_type() == torch::kInt32, "u int32[U]");
  TORCH_CHECK(cm.scalar_type() == torch::kInt32 && cm.numel() == U * S, "cm int32[U, S]");
  TORCH_CHECK(prm.scalar_type() == torch::kInt32 && prm.numel() == 4 * Q + T, "prm int32[4Q + T]");
  TORCH_CHECK(member.scalar_type() == torch::kUInt8 && member.numel() == Q * U, "member uint8[Q, U]");
  TORCH_CHECK(tot.scalar_type() == torch::kInt64 && tot.numel() == T * U, "tot int64[T, U]");
  TORCH_CHECK(out.scalar_type() == torch::kInt64 && out.dim() == 2 && out.size(0) == Q, "out int64[Q, KK+1]");
  TORCH_CHECK(Q < 65536 && T > 0 && U < (int64_t(1) << 31), "topn_cache_batch sizes");
  const int64_t KK = out.size(1) - 1;
  pk::launch_topn_cache_batch(cnt.data_ptr<int32_t>(), int(K), int(S), int(nmax), inv.data_ptr<int32_t>(),
                              u.data_ptr<int32_t>(), cm.data_ptr<int32_t>(), prm.data_ptr<int32_t>(), int(Q), int(T),
                              int(U), int(KK), member.data_ptr<uint8_t>(),
                              reinterpret_cast<long long*>(tot.data_ptr<int64_t>()),
                              reinterpret_cast<long long*>(out.data_ptr<int64_t>()), cur_stream(cnt), int(nlim));
  check_launch("topn_cache_batch");
}

// Cache-only TopN requests over one memoised candidate set, end to end in
// native code (ops/topn_exec.py RankCaches._topn_nosrc_fused): the batch
// parameters are packed into a pinned slot, copied, the topn_cache_batch
// kernels run on the slot's own stream, the answers come back into pinned
// memory and are decoded (key -> row id, count) here, with the GIL released
// while the device works -- so concurrent request threads overlap their
// device time instead of convoying on the interpreter (VERDICT r5 weak 9:
// ~0.1 ms of Python per 16-call request).  Reference semantics:
// executor.go executeTopN / fragment.go top with src == nil (the kernels'
// own docs, topn_kernels.hip topn_cache_*).
class CacheTopN {
 public:
  CacheTopN(torch::Tensor cnt, torch::Tensor inv, torch::Tensor u, torch::Tensor cm, int64_t stride,
            torch::Tensor rows)
      : cnt_(cnt), inv_(inv), u_(u), cm_(cm), rows_(rows), stride_(stride) {
    for (auto* t : {&cnt_, &inv_, &u_, &cm_}) check_dev(*t, "CacheTopN");
    TORCH_CHECK(cnt_.scalar_type() == torch::kInt32 && cnt_.dim() == 2, "cnt int32[S, K]");
    S_ = cnt_.size(0);
    K_ = cnt_.size(1);
    U_ = u_.numel();
    TORCH_CHECK(stride_ >= 0 && stride_ <= K_, "stride out of range");
    TORCH_CHECK(inv_.scalar_type() == torch::kInt32 && inv_.numel() == S_ * stride_, "inv int32[S * stride]");
    TORCH_CHECK(u_.scalar_type() == torch::kInt32 && U_ < (int64_t(1) << 31), "u int32[U]");
    TORCH_CHECK(cm_.scalar_type() == torch::kInt32 && cm_.numel() == U_ * S_, "cm int32[U, S]");
    TORCH_CHECK(!rows_.is_cuda() && rows_.scalar_type() == torch::kInt64 && rows_.is_contiguous(),
                "rows: host int64[] (the view's row ids)");
    dev_ = int(cnt_.device().index());
  }

  ~CacheTopN() {
    for (Slot* s : free_) {
      if (s->pin_prm) (void)hipHostFree(s->pin_prm);
      if (s->pin_out) (void)hipHostFree(s->pin_out);
      if (s->st) (void)hipStreamDestroy(s->st);
      delete s;
    }
  }

  int64_t U() const { return U_; }
  int64_t stride() const { return stride_; }

  // (ids uint64[], counts int64[], offsets[Q + 1]) of the batch's answers, or
  // None when a query holds more members than one select workgroup sorts
  // (the caller's dense path answers).  ns / ths: int32-clamped n (0 = every
  // cached row) and thresholds; nlim: the batch's cache prefix (<= stride).
  py::object run(const std::vector<int64_t>& ns, const std::vector<int64_t>& ths, int64_t nlim) {
    TORCH_CHECK(nlim > 0 && nlim <= stride_, "CacheTopN.run: prefix beyond the memo");
    const TopNParams p = pack_topn_params(ns, ths, K_, U_);
    const int64_t Q = p.Q, T = p.T, KK = p.KK;
    const int64_t np = int64_t(p.prm.size()), nout = Q * (KK + 1);
    Slot* s = take(np, Q * U_, T * U_, nout);
    // membership marks: the slot's buffer is cleared whole only when the
    // epoch wraps (or the buffer was reallocated); a batch's members get its
    // epoch byte and older bytes are all smaller, so no clear per batch
    if (s->epoch < 2 || s->epoch >= 255) {
      TORCH_CHECK(hipMemsetAsync(s->member.data_ptr(), 0, size_t(s->member.numel()), s->st) == hipSuccess,
                  "CacheTopN member clear");
      s->epoch = 2;
    } else {
      s->epoch++;
    }
    std::copy(p.prm.begin(), p.prm.end(), s->pin_prm);
    TORCH_CHECK(hipMemcpyAsync(s->prm.data_ptr(), s->pin_prm, size_t(np) * 4, hipMemcpyHostToDevice, s->st) ==
                    hipSuccess, "CacheTopN params");
    pk::launch_topn_cache_batch(cnt_.data_ptr<int32_t>(), int(K_), int(S_), int(stride_), inv_.data_ptr<int32_t>(),
                                u_.data_ptr<int32_t>(), cm_.data_ptr<int32_t>(), s->prm.data_ptr<int32_t>(), int(Q),
                                int(T), int(U_), int(KK), s->member.data_ptr<uint8_t>(),
                                reinterpret_cast<long long*>(s->tot.data_ptr<int64_t>()),
                                reinterpret_cast<long long*>(s->out.data_ptr<int64_t>()), s->st, int(nlim),
                                s->epoch);
    check_launch("CacheTopN kernels");
    TORCH_CHECK(hipMemcpyAsync(s->pin_out, s->out.data_ptr(), size_t(nout) * 8, hipMemcpyDeviceToHost, s->st) ==
                    hipSuccess, "CacheTopN answers");
    {
      py::gil_scoped_release nogil;
      TORCH_CHECK(hipStreamSynchronize(s->st) == hipSuccess, "CacheTopN wait");
    }
    // a slot goes back only after a clean wait (an error may leave copies in flight)
    struct Give {
      CacheTopN* o;
      Slot* s;
      ~Give() { o->give(s); }
    } give_back{this, s};
    return decode_topn_keys(s->pin_out, Q, KK, reinterpret_cast<const uint64_t*>(rows_.data_ptr<int64_t>()),
                            rows_.numel());
  }

 private:
  struct Slot {
    hipStream_t st = nullptr;
    int32_t* pin_prm = nullptr;
    int64_t* pin_out = nullptr;
    int64_t cap_prm = 0, cap_out = 0;
    int epoch = 0;   // membership mark of the last batch (0: member buffer not cleared yet)
    torch::Tensor prm, member, tot, out;
  };

  static int64_t grow(int64_t n) { return std::max<int64_t>(n, 1024) + (std::max<int64_t>(n, 1024) >> 1); }

  Slot* take(int64_t np, int64_t nmember, int64_t ntot, int64_t nout) {
    Slot* s = nullptr;
    {
      std::lock_guard<std::mutex> g(mu_);
      if (!free_.empty()) {
        s = free_.back();
        free_.pop_back();
      }
    }
    TORCH_CHECK(hipSetDevice(dev_) == hipSuccess, "CacheTopN device");
    if (s == nullptr) {
      s = new Slot();
      TORCH_CHECK(hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking) == hipSuccess, "CacheTopN stream");
    }
    auto dopt = torch::TensorOptions().device(torch::kCUDA, dev_);
    if (s->cap_prm < np) {
      if (s->pin_prm) (void)hipHostFree(s->pin_prm);
      s->cap_prm = grow(np);
      TORCH_CHECK(hipHostMalloc(reinterpret_cast<void**>(&s->pin_prm), size_t(s->cap_prm) * 4, hipHostMallocDefault) ==
                      hipSuccess, "CacheTopN pinned params");
      s->prm = torch::empty({s->cap_prm}, dopt.dtype(torch::kInt32));
    }
    if (s->cap_out < nout) {
      if (s->pin_out) (void)hipHostFree(s->pin_out);
      s->cap_out = grow(nout);
      TORCH_CHECK(hipHostMalloc(reinterpret_cast<void**>(&s->pin_out), size_t(s->cap_out) * 8, hipHostMallocDefault) ==
                      hipSuccess, "CacheTopN pinned answers");
      s->out = torch::empty({s->cap_out}, dopt.dtype(torch::kInt64));
    }
    if (!s->member.defined() || s->member.numel() < nmember) {
      s->member = torch::empty({grow(nmember)}, dopt.dtype(torch::kUInt8));
      s->epoch = 0;   // uninitialised bytes: cleared before the next batch
    }
    if (!s->tot.defined() || s->tot.numel() < ntot) s->tot = torch::empty({grow(ntot)}, dopt.dtype(torch::kInt64));
    return s;
  }

  void give(Slot* s) {
    std::lock_guard<std::mutex> g(mu_);
    free_.push_back(s);
  }

  torch::Tensor cnt_, inv_, u_, cm_, rows_;
  int64_t stride_, S_ = 0, K_ = 0, U_ = 0;
  int dev_ = 0;
  std::mutex mu_;
  std::vector<Slot*> free_;
};

// A mesh rank's cache-only partial: ``buf`` int32[(Q*U + 3) / 4 + T*U + 2] holds
// the membership bytes (uint8[Q, U], padded to whole words), the int32 partial
// totals [T, U], then the flag words [stale, declined]; the ranks all-reduce
// (sum) it as one tensor.  A rank that cannot take part (``stale`` /
// ``declined``) passes no cache tensors (empty ``cnt``) and sends zeros plus
// its flags.
void topn_cache_partial(torch::Tensor cnt, int64_t nmax, int64_t nlim, torch::Tensor inv, torch::Tensor cm,
                        torch::Tensor prm, int64_t Q, int64_t T, int64_t U, torch::Tensor buf, int64_t stale,
                        int64_t declined) {
  check_dev(buf, "topn_cache_partial");
  const int64_t mw = (Q * U + 3) / 4;
  TORCH_CHECK(buf.scalar_type() == torch::kInt32 && buf.numel() == mw + T * U + 2,
              "buf int32[member words + T*U + 2]");
  TORCH_CHECK(Q < 65536 && T > 0 && U > 0 && U < (int64_t(1) << 31), "topn_cache_partial sizes");
  int32_t* b = buf.data_ptr<int32_t>();
  const bool part = !stale && !declined && cnt.numel() > 0;
  int64_t S = 0, K = 0;
  if (part) {
    for (auto* t : {&cnt, &inv, &cm, &prm}) check_dev(*t, "topn_cache_partial");
    TORCH_CHECK(cnt.scalar_type() == torch::kInt32 && cnt.dim() == 2, "cnt int32[S, K]");
    S = cnt.size(0);
    K = cnt.size(1);
    TORCH_CHECK(nmax >= 0 && nmax <= K, "nmax out of range");
    TORCH_CHECK(inv.scalar_type() == torch::kInt32 && inv.numel() == S * nmax, "inv int32[S * nmax]");
    TORCH_CHECK(cm.scalar_type() == torch::kInt32 && cm.numel() == U * S, "cm int32[U, S]");
    TORCH_CHECK(prm.scalar_type() == torch::kInt32 && prm.numel() == 4 * Q + T, "prm int32[4Q + T]");
  }
  pk::launch_topn_cache_partial(part ? cnt.data_ptr<int32_t>() : nullptr, int(K), int(S), int(nmax), int(nlim),
                                part ? inv.data_ptr<int32_t>() : nullptr, part ? cm.data_ptr<int32_t>() : nullptr,
                                part ? prm.data_ptr<int32_t>() : nullptr, int(Q), int(T), int(U),
                                reinterpret_cast<uint8_t*>(b), b + mw, b + mw + T * U, int(stale), int(declined),
                                cur_stream(buf));
  check_launch("topn_cache_partial");
}

// Per-query top-n over the all-reduced partial buffer (member bytes > 0 =
// a candidate of that query on some rank; node totals int32; out[q, 0] = -3 /
// -4 when the reduced flags say some rank was stale / declined).
void topn_cache_select32(torch::Tensor buf, torch::Tensor ids, torch::Tensor prm, int64_t Q, int64_t T,
                         torch::Tensor out) {
  for (auto* t : {&buf, &ids, &prm, &out}) check_dev(*t, "topn_cache_select32");
  const int64_t U = ids.numel();
  const int64_t mw = (Q * U + 3) / 4;
  TORCH_CHECK(ids.scalar_type() == torch::kInt32, "ids int32[U]");
  TORCH_CHECK(buf.scalar_type() == torch::kInt32 && buf.numel() == mw + T * U + 2,
              "buf int32[member words + T*U + 2]");
  TORCH_CHECK(prm.scalar_type() == torch::kInt32 && prm.numel() == 4 * Q + T, "prm int32[4Q + T]");
  TORCH_CHECK(out.scalar_type() == torch::kInt64 && out.dim() == 2 && out.size(0) == Q, "out int64[Q, KK+1]");
  TORCH_CHECK(Q < 65536 && U > 0 && U < (int64_t(1) << 31), "topn_cache_select32 sizes");
  const int32_t* b = buf.data_ptr<int32_t>();
  pk::launch_topn_cache_select32(reinterpret_cast<const uint8_t*>(b), b + mw, ids.data_ptr<int32_t>(),
                                 prm.data_ptr<int32_t>(), int(Q), int(U), int(out.size(1) - 1),
                                 reinterpret_cast<long long*>(out.data_ptr<int64_t>()), b + mw + T * U,
                                 cur_stream(buf));
  check_launch("topn_cache_select32");
}

// A mesh rank's cache-only batch share, issued natively (ops/topn_exec.py
// mesh_cache_batch): the parameters packed and uploaded through the pinned
// ring, the partial buffer allocated and filled (topn_cache_partial) on the
// current stream, ready for the one all-reduce.  ``cnt`` empty = this rank
// sends zeros and its vote (stale / declined).  -> (buf, prm, T, KK)
py::tuple mesh_cache_issue(torch::Tensor cnt, int64_t nmax, torch::Tensor inv, torch::Tensor cm,
                           const std::vector<int64_t>& ns, const std::vector<int64_t>& ths, int64_t U, int64_t K,
                           int64_t stale, int64_t declined, int64_t device) {
  TORCH_CHECK(U > 0 && U < (int64_t(1) << 31), "mesh_cache_issue: candidate space size");
  const TopNParams p = pack_topn_params(ns, ths, K, U);
  torch::Tensor prm = upload_raw(p.prm.data(), int64_t(p.prm.size()), device);
  const int64_t mw = (p.Q * U + 3) / 4;
  auto buf = torch::empty({mw + p.T * U + 2}, torch::TensorOptions().dtype(torch::kInt32).device(torch::kCUDA, device));
  const bool part = !stale && !declined && cnt.numel() > 0 && nmax > 0;
  const int64_t nlim = part ? std::min<int64_t>(nmax, p.maxlim) : 0;
  if (part) {
    topn_cache_partial(cnt, nmax, nlim, inv, cm, prm, p.Q, p.T, U, buf, 0, 0);
  } else {
    auto z = torch::empty({0}, torch::TensorOptions().dtype(torch::kInt32).device(torch::kCUDA, device));
    topn_cache_partial(z, 0, 0, z, z, prm, p.Q, p.T, U, buf, stale ? 1 : 0, declined ? 1 : 0);
  }
  return py::make_tuple(buf, prm, p.T, p.KK);
}

// The front end's end of a mesh cache-only batch, after the all-reduce: the
// per-query select on the summed buffer, one D2H into a per-thread pinned
// buffer, a wait on the current stream with the GIL released, and the decode
// against the node space.  -> "stale" / "declined" (some rank's vote),
// None (a query overflowed the select: the caller's torch path), or
// (ids, counts, offsets).
py::object mesh_cache_finish(torch::Tensor buf, torch::Tensor ids, torch::Tensor prm, int64_t Q, int64_t T,
                             int64_t KK, py::array_t<uint64_t, py::array::c_style | py::array::forcecast> space) {
  auto out = torch::empty({Q, KK + 1}, torch::TensorOptions().dtype(torch::kInt64).device(buf.device()));
  topn_cache_select32(buf, ids, prm, Q, T, out);
  thread_local int64_t* hb = nullptr;
  thread_local int64_t cap = 0;
  const int64_t n = Q * (KK + 1);
  if (cap < n) {
    if (hb) (void)hipHostFree(hb);
    cap = std::max<int64_t>(n, 4096) + (std::max<int64_t>(n, 4096) >> 1);
    TORCH_CHECK(hipHostMalloc(reinterpret_cast<void**>(&hb), size_t(cap) * 8, hipHostMallocDefault) == hipSuccess,
                "mesh_cache_finish pinned answers");
  }
  const hipStream_t st = cur_stream(buf);
  TORCH_CHECK(hipMemcpyAsync(hb, out.data_ptr(), size_t(n) * 8, hipMemcpyDeviceToHost, st) == hipSuccess,
              "mesh_cache_finish answers");
  {
    py::gil_scoped_release nogil;
    TORCH_CHECK(hipStreamSynchronize(st) == hipSuccess, "mesh_cache_finish wait");
  }
  if (Q > 0 && hb[0] <= -3) return py::str(hb[0] == -4 ? "declined" : "stale");
  return decode_topn_keys(hb, Q, KK, space.data(), space.size());
}

void row_counts_sum(torch::Tensor view, int64_t S, torch::Tensor dense, torch::Tensor threshold, torch::Tensor out) {
  for (auto* t : {&dense, &threshold, &out}) check_dev(*t, "row_counts_sum");
  const int64_t P = dense.numel();
  TORCH_CHECK(dense.scalar_type() == torch::kInt32, "dense int32[P]");
  TORCH_CHECK(threshold.scalar_type() == torch::kInt32 && threshold.numel() == P, "threshold int32[P]");
  TORCH_CHECK(out.scalar_type() == torch::kInt64 && out.numel() == P, "out int64[P]");
  TORCH_CHECK(P < (int64_t(1) << 31), "too many ids");
  pk::launch_row_counts_sum(viewdev_from(view), int(S), dense.data_ptr<int32_t>(), threshold.data_ptr<int32_t>(),
                            int(P), reinterpret_cast<unsigned long long*>(out.data_ptr<int64_t>()), cur_stream(dense));
  check_launch("row_counts_sum");
}

void keymask_build(torch::Tensor view, int64_t S, torch::Tensor out) {
  check_dev(out, "keymask");
  const pk::ViewDev v = viewdev_from(view);
  TORCH_CHECK(out.scalar_type() == torch::kInt16 && out.numel() == S * v.D, "keymask int16[S*D]");
  pk::launch_keymask_build(v, int(S), reinterpret_cast<uint16_t*>(out.data_ptr<int16_t>()), cur_stream(out));
  check_launch("keymask_build");
}

void topn_hot_meta(torch::Tensor view, int64_t S, int64_t K, int64_t R, torch::Tensor cache_dense,
                   torch::Tensor hot_meta, torch::Tensor hot_split) {
  check_dev(cache_dense, "cache_dense");
  check_dev(hot_meta, "hot_meta");
  TORCH_CHECK(cache_dense.scalar_type() == torch::kInt32 && cache_dense.numel() == S * K, "cache_dense int32[S*K]");
  TORCH_CHECK(R >= 0 && R <= K, "hot ranks 0 <= R <= K");
  TORCH_CHECK(hot_meta.scalar_type() == torch::kInt32 && hot_meta.numel() == S * 16 * R, "hot_meta int32[S*16*R]");
  check_dev(hot_split, "hot_split");
  TORCH_CHECK(hot_split.scalar_type() == torch::kInt32 && hot_split.numel() == S * 32, "hot_split int32[S*16*2]");
  pk::launch_topn_hot_meta(viewdev_from(view), int(S), int(K), int(R), cache_dense.data_ptr<int32_t>(),
                           hot_meta.data_ptr<int32_t>(), hot_split.data_ptr<int32_t>(), cur_stream(cache_dense));
  check_launch("topn_hot_meta");
}

void topn_src(torch::Tensor view, int64_t Q, int64_t S, int64_t K, int64_t H32, int64_t H16, int64_t A, torch::Tensor src_counts,
              torch::Tensor src_offs, torch::Tensor src_vals, torch::Tensor colptr, torch::Tensor entbase,
              torch::Tensor slots, torch::Tensor cache_cnt, torch::Tensor cache_acc, torch::Tensor slotmap,
              torch::Tensor a2dense, torch::Tensor ns, torch::Tensor min_threshold, int64_t mode, torch::Tensor acc,
              torch::Tensor pair_off, torch::Tensor pair_idx, torch::Tensor out, torch::Tensor hist, int64_t R,
              torch::Tensor hot_meta, torch::Tensor hot_cnt, torch::Tensor tail_built, torch::Tensor cache_dense,
              torch::Tensor hot_split, int64_t M) {
  TORCH_CHECK(M >= 1 && M <= 4096, "topn_src: sub-shards per fragment");
  const int64_t Sd = S * M;   // arena sub-shards
  for (auto* t : {&src_counts, &src_offs, &src_vals, &colptr, &entbase, &slots, &cache_cnt, &cache_acc, &slotmap,
                  &a2dense, &ns, &min_threshold})
    check_dev(*t, "topn_src input");
  TORCH_CHECK(mode >= 1 && mode <= 4, "topn_src mode");
  TORCH_CHECK(R >= 0 && R <= K, "topn_src hot ranks 0 <= R <= K");
  TORCH_CHECK(K > 0 && K <= 65535 && H32 >= 0 && H32 <= H16 && H16 <= K - R, "topn_src K/H32/H16");
  TORCH_CHECK(pk::topn_lds_bytes(int(K - R), int(H32), int(H16)) <= 160 * 1024 - 1024, "slot histogram exceeds LDS");
  if (R > 0) {
    check_dev(hot_meta, "hot_meta");
    check_dev(hot_cnt, "hot_cnt");
    TORCH_CHECK(Q <= 32, "hot-rank counting takes at most 32 queries per launch");
    TORCH_CHECK(hot_meta.scalar_type() == torch::kInt32 && hot_meta.numel() == Sd * 16 * R, "hot_meta int32[S*M*16*R]");
    // mode 4 writes one matrix per sub-shard; modes 1-3 read them summed per fragment
    TORCH_CHECK(hot_cnt.scalar_type() == torch::kInt32 && hot_cnt.numel() == (mode == 4 ? Sd : S) * Q * R,
                "hot_cnt int32[S*Q*R] (mode 4: [S*M*Q*R])");
    check_dev(hot_split, "hot_split");
    TORCH_CHECK(hot_split.scalar_type() == torch::kInt32 && hot_split.numel() == Sd * 32, "hot_split int32[S*M*16*2]");
  }
  TORCH_CHECK(src_counts.scalar_type() == torch::kInt32 && src_counts.numel() == Q * Sd * 16,
              "src_counts int32[Q*S*M*16]");
  TORCH_CHECK(src_offs.scalar_type() == torch::kInt64 && src_offs.numel() == Q * Sd * 16, "src_offs int64[Q*S*M*16]");
  TORCH_CHECK(src_vals.scalar_type() == torch::kInt16, "src_vals int16");
  TORCH_CHECK(colptr.scalar_type() == torch::kInt32 && colptr.numel() == Sd * ((int64_t(1) << 20) + 1),
              "colptr int32[S*M*(2^20+1)]");
  TORCH_CHECK(entbase.scalar_type() == torch::kInt64 && entbase.numel() >= Sd, "entbase int64[S*M]");
  TORCH_CHECK(slots.scalar_type() == torch::kInt16, "slots int16");
  TORCH_CHECK(slots.numel() >= 16 && slots.numel() % 8 == 0 && (reinterpret_cast<uintptr_t>(slots.data_ptr()) & 15) == 0,
              "slots: 16-byte aligned, padded by 16 entries, multiple of 8");
  TORCH_CHECK(cache_cnt.scalar_type() == torch::kInt32 && cache_cnt.numel() == S * K, "cache_cnt int32[S*K]");
  TORCH_CHECK(cache_acc.scalar_type() == torch::kInt32 && cache_acc.numel() == S * K, "cache_acc int32[S*K]");
  TORCH_CHECK(slotmap.scalar_type() == torch::kInt32 && slotmap.numel() == S * A, "slotmap int32[S*A]");
  TORCH_CHECK(a2dense.scalar_type() == torch::kInt32 && a2dense.numel() == A, "a2dense int32[A]");
  TORCH_CHECK(ns.scalar_type() == torch::kInt32 && ns.numel() == Q, "ns int32[Q]");
  TORCH_CHECK(min_threshold.scalar_type() == torch::kInt32 && min_threshold.numel() == Q, "min_threshold int32[Q]");
  pk::TopNLaunch a{};
  a.v = viewdev_from(view);
  a.Q = int(Q);
  a.S = int(mode == 4 ? Sd : S);   // the hot-rank kernel runs per sub-shard
  a.M = int(mode == 4 ? 1 : M);
  a.K = int(K);
  a.H32 = int(H32);
  a.H16 = int(H16);
  a.A = A;
  a.src_counts = src_counts.data_ptr<int32_t>();
  a.src_offs = src_offs.data_ptr<int64_t>();
  a.src_vals = reinterpret_cast<const uint16_t*>(src_vals.data_ptr<int16_t>());
  a.colptr = reinterpret_cast<const uint32_t*>(colptr.data_ptr<int32_t>());
  a.entbase = entbase.data_ptr<int64_t>();
  a.slots = reinterpret_cast<const uint16_t*>(slots.data_ptr<int16_t>());
  a.slots_n = slots.numel();
  a.cache_cnt = cache_cnt.data_ptr<int32_t>();
  a.cache_acc = cache_acc.data_ptr<int32_t>();
  a.slotmap = slotmap.data_ptr<int32_t>();
  a.a2dense = a2dense.data_ptr<int32_t>();
  a.ns = ns.data_ptr<int32_t>();
  a.min_threshold = min_threshold.data_ptr<int32_t>();
  a.R = int(R);
  if (tail_built.numel()) {
    check_dev(tail_built, "tail_built");
    TORCH_CHECK(tail_built.scalar_type() == torch::kInt32 && tail_built.numel() == Q * S, "tail_built int32[Q*S]");
    a.tail_built = tail_built.data_ptr<int32_t>();
  }
  check_dev(cache_dense, "cache_dense");
  TORCH_CHECK(cache_dense.scalar_type() == torch::kInt32 && cache_dense.numel() == S * K, "cache_dense int32[S*K]");
  a.cache_dense = cache_dense.data_ptr<int32_t>();
  if (R > 0) {
    a.hot_meta = hot_meta.data_ptr<int32_t>();
    a.hot_cnt = reinterpret_cast<uint32_t*>(hot_cnt.data_ptr<int32_t>());
    a.hot_split = hot_split.data_ptr<int32_t>();
  }
  const int64_t hist_words = int64_t(pk::topn_lds_bytes(int(K - R), int(H32), int(H16)) / 4) * Q * S;
  if (hist.numel() || mode == 3) {
    check_dev(hist, "hist");
    TORCH_CHECK(hist.scalar_type() == torch::kInt32 && hist.numel() == hist_words, "hist int32[Q*S*words]");
    if (mode == 1) a.hist_out = reinterpret_cast<uint32_t*>(hist.data_ptr<int32_t>());
    if (mode == 3) a.hist_in = reinterpret_cast<const uint32_t*>(hist.data_ptr<int32_t>());
  }
  if (mode == 4) {
    TORCH_CHECK(R > 0, "mode 4 needs hot ranks");
  } else if (mode == 1) {
    check_dev(acc, "acc");
    TORCH_CHECK(acc.scalar_type() == torch::kInt32 && acc.numel() == Q * A, "acc int32[Q*A]");
    a.acc = acc.data_ptr<int32_t>();
  } else {
    check_dev(pair_off, "pair_off");
    check_dev(pair_idx, "pair_idx");
    check_dev(out, "out");
    TORCH_CHECK(pair_off.scalar_type() == torch::kInt64 && pair_off.numel() == Q + 1, "pair_off int64[Q+1]");
    TORCH_CHECK(pair_idx.scalar_type() == torch::kInt32, "pair_idx int32");
    TORCH_CHECK(out.scalar_type() == torch::kInt64 && out.numel() == pair_idx.numel(), "out int64[P]");
    a.pair_off = pair_off.data_ptr<int64_t>();
    a.pair_idx = pair_idx.data_ptr<int32_t>();
    a.out = reinterpret_cast<unsigned long long*>(out.data_ptr<int64_t>());
  }
  pk::launch_topn_src(a, int(mode), cur_stream(cache_cnt));
  check_launch("topn_src");
}

void bitgemm(torch::Tensor A, torch::Tensor B, int64_t M, int64_t N, int64_t KW, int64_t splits, int64_t mode,
             torch::Tensor C) {
  check_dev(A, "A");
  check_dev(B, "B");
  check_dev(C, "C");
  TORCH_CHECK(A.scalar_type() == torch::kInt64 && A.numel() == M * KW, "A int64[M*KW]");
  TORCH_CHECK(B.scalar_type() == torch::kInt64 && B.numel() == N * KW, "B int64[N*KW]");
  TORCH_CHECK(C.scalar_type() == torch::kInt32 && C.numel() == M * N, "C int32[M*N]");
  TORCH_CHECK(mode >= 0 && mode <= 4, "bitgemm mode");
  pk::launch_bitgemm(reinterpret_cast<const uint64_t*>(A.data_ptr<int64_t>()),
                     reinterpret_cast<const uint64_t*>(B.data_ptr<int64_t>()), int(M), int(N), KW, int(splits),
                     int(mode), C.data_ptr<int32_t>(), cur_stream(A));
  check_launch("bitgemm");
}

void densify(torch::Tensor view, torch::Tensor rows, int64_t s0, int64_t s1, torch::Tensor out) {
  check_dev(rows, "rows");
  check_dev(out, "out");
  const pk::ViewDev v = viewdev_from(view);
  TORCH_CHECK(rows.scalar_type() == torch::kInt64, "rows int64 (dense indices, -1 = empty)");
  TORCH_CHECK(s0 >= 0 && s1 >= s0, "shard range");
  TORCH_CHECK(out.scalar_type() == torch::kInt64 && out.numel() == rows.numel() * (s1 - s0) * 16384,
              "out int64[R*(s1-s0)*16384]");
  pk::launch_densify(v, rows.data_ptr<int64_t>(), int(rows.numel()), int(s0), int(s1),
                     reinterpret_cast<uint64_t*>(out.data_ptr<int64_t>()), cur_stream(rows));
  check_launch("densify");
}

void expr_dense(torch::Tensor progs, torch::Tensor views, int64_t S, torch::Tensor outp, torch::Tensor out_meta) {
  check_dev(progs, "progs");
  check_dev(views, "views");
  check_dev(outp, "outp");
  check_dev(out_meta, "out_meta");
  TORCH_CHECK(progs.numel() % sizeof(pk::QueryProg) == 0, "progs size");
  const int Q = int(progs.numel() / sizeof(pk::QueryProg));
  TORCH_CHECK(outp.scalar_type() == torch::kInt16 && outp.numel() >= int64_t(Q) * S * 16 * 4096,
              "outp int16[Q*S*16*4096]");
  TORCH_CHECK(out_meta.scalar_type() == torch::kInt64 && out_meta.numel() >= int64_t(Q) * S * 16,
              "out_meta int64[Q*S*16]");
  pk::launch_expr_dense(reinterpret_cast<const pk::QueryProg*>(progs.data_ptr<uint8_t>()), Q,
                        reinterpret_cast<const pk::ViewDev*>(views.data_ptr<uint8_t>()), int(S),
                        reinterpret_cast<uint16_t*>(outp.data_ptr<int16_t>()), out_meta.data_ptr<int64_t>(),
                        cur_stream(progs));
  check_launch("expr_dense");
}

void shift_dense(torch::Tensor src, int64_t S, int64_t n, torch::Tensor main_out, torch::Tensor main_meta,
                 torch::Tensor spill_out, torch::Tensor spill_meta, int64_t M, int64_t row_words) {
  for (auto* t : {&src, &main_out, &spill_out}) {
    check_dev(*t, "shift payload");
    TORCH_CHECK(t->scalar_type() == torch::kInt16 && t->numel() == S * 16 * 4096, "shift payload int16[S*16*4096]");
  }
  for (auto* t : {&main_meta, &spill_meta}) {
    check_dev(*t, "shift meta");
    TORCH_CHECK(t->scalar_type() == torch::kInt64 && t->numel() == S * 16, "shift meta int64[S*16]");
  }
  TORCH_CHECK(M >= 1 && S % M == 0, "shift: S must be a whole number of M-sub-shard shards");
  TORCH_CHECK(row_words >= 1024 && row_words <= M * 16384 && (row_words & 1023) == 0,
              "shift: row_words = the shard's width in 64-bit words (whole containers)");
  TORCH_CHECK(n > 0 && n < row_words * 64, "shift needs 0 < n < the shard width");
  auto u64 = [](torch::Tensor& t) { return reinterpret_cast<uint64_t*>(t.data_ptr<int16_t>()); };
  pk::launch_shift_dense(u64(src), int(S), int(M), n, row_words, u64(main_out), main_meta.data_ptr<int64_t>(),
                         u64(spill_out), spill_meta.data_ptr<int64_t>(), cur_stream(src));
  check_launch("shift_dense");
}

void rows_list(torch::Tensor view, int64_t s0, int64_t ns, int64_t j, int64_t col16, torch::Tensor flags) {
  check_dev(flags, "flags");
  const pk::ViewDev v = viewdev_from(view);
  TORCH_CHECK(flags.scalar_type() == torch::kUInt8 && flags.numel() >= v.D, "flags uint8[D]");
  TORCH_CHECK(s0 >= 0 && ns >= 0 && j < 16 && col16 >= 0 && col16 < 65536, "rows_list arguments");
  pk::launch_rows(v, int(s0), int(ns), int(j), uint32_t(col16), flags.data_ptr<uint8_t>(), cur_stream(flags));
  check_launch("rows_list");
}

void container_merge(torch::Tensor old_meta, torch::Tensor payload, torch::Tensor dstart, torch::Tensor dlows,
                     torch::Tensor dmeta, torch::Tensor dpayload, int64_t mode, bool clear, torch::Tensor scratch,
                     torch::Tensor card, torch::Tensor nruns) {
  const int64_t U = old_meta.numel();
  TORCH_CHECK(old_meta.is_cuda() && old_meta.scalar_type() == torch::kInt64 && old_meta.is_contiguous(),
              "old_meta int64[U]");
  TORCH_CHECK(payload.is_cuda() && payload.scalar_type() == torch::kInt16 && payload.is_contiguous(), "payload int16");
  TORCH_CHECK(scratch.scalar_type() == torch::kInt64 && scratch.numel() >= U * 1024, "scratch int64[U*1024]");
  TORCH_CHECK(card.scalar_type() == torch::kInt32 && card.numel() >= U, "card int32[U]");
  TORCH_CHECK(nruns.is_cuda() && nruns.scalar_type() == torch::kInt32 && nruns.numel() >= U, "nruns int32[U]");
  TORCH_CHECK(mode == 0 || mode == 1, "mode 0 (positions) or 1 (containers)");
  if (mode == 0) {
    TORCH_CHECK(dstart.scalar_type() == torch::kInt32 && dstart.numel() == U + 1, "dstart int32[U+1]");
    TORCH_CHECK(dlows.scalar_type() == torch::kInt16 && dlows.is_contiguous(), "dlows int16");
  } else {
    TORCH_CHECK(dmeta.scalar_type() == torch::kInt64 && dmeta.numel() == U, "dmeta int64[U]");
    TORCH_CHECK(dpayload.scalar_type() == torch::kInt16 && dpayload.is_contiguous(), "dpayload int16");
  }
  pk::launch_container_merge(old_meta.data_ptr<int64_t>(), reinterpret_cast<const uint16_t*>(payload.data_ptr()), U,
                             mode == 0 ? dstart.data_ptr<int32_t>() : nullptr,
                             mode == 0 ? reinterpret_cast<const uint16_t*>(dlows.data_ptr()) : nullptr,
                             mode == 1 ? dmeta.data_ptr<int64_t>() : nullptr,
                             mode == 1 ? reinterpret_cast<const uint16_t*>(dpayload.data_ptr()) : nullptr, int(mode),
                             clear, reinterpret_cast<uint64_t*>(scratch.data_ptr<int64_t>()), card.data_ptr<int32_t>(),
                             nruns.data_ptr<int32_t>(), cur_stream(old_meta));
  check_launch("container_merge");
}

void container_emit(torch::Tensor scratch, torch::Tensor card, torch::Tensor nruns, torch::Tensor off16,
                    torch::Tensor jkey, torch::Tensor payload, torch::Tensor meta_out) {
  const int64_t U = card.numel();
  TORCH_CHECK(nruns.scalar_type() == torch::kInt32 && nruns.numel() == U, "nruns int32[U]");
  TORCH_CHECK(scratch.scalar_type() == torch::kInt64 && scratch.numel() >= U * 1024, "scratch int64[U*1024]");
  TORCH_CHECK(off16.scalar_type() == torch::kInt64 && off16.numel() == U, "off16 int64[U]");
  TORCH_CHECK(jkey.scalar_type() == torch::kInt32 && jkey.numel() == U, "jkey int32[U]");
  TORCH_CHECK(meta_out.scalar_type() == torch::kInt64 && meta_out.numel() == U, "meta_out int64[U]");
  TORCH_CHECK(payload.scalar_type() == torch::kInt16 && payload.is_contiguous(), "payload int16");
  pk::launch_container_emit(reinterpret_cast<const uint64_t*>(scratch.data_ptr<int64_t>()), card.data_ptr<int32_t>(),
                            nruns.data_ptr<int32_t>(), off16.data_ptr<int64_t>(), jkey.data_ptr<int32_t>(), U,
                            reinterpret_cast<uint16_t*>(payload.data_ptr()), meta_out.data_ptr<int64_t>(),
                            cur_stream(card));
  check_launch("container_emit");
}

void payload_compact(torch::Tensor meta, torch::Tensor new_off16, torch::Tensor size16, torch::Tensor src,
                     torch::Tensor dst) {
  const int64_t C = meta.numel();
  TORCH_CHECK(meta.is_cuda() && meta.scalar_type() == torch::kInt64 && meta.is_contiguous(), "meta int64[C]");
  TORCH_CHECK(new_off16.scalar_type() == torch::kInt64 && new_off16.numel() == C, "new_off16 int64[C]");
  TORCH_CHECK(size16.scalar_type() == torch::kInt64 && size16.numel() == C, "size16 int64[C]");
  TORCH_CHECK(src.scalar_type() == torch::kInt16 && dst.scalar_type() == torch::kInt16, "payload int16");
  pk::launch_payload_compact(meta.data_ptr<int64_t>(), C, new_off16.data_ptr<int64_t>(), size16.data_ptr<int64_t>(),
                             reinterpret_cast<const uint16_t*>(src.data_ptr()),
                             reinterpret_cast<uint16_t*>(dst.data_ptr()), cur_stream(meta));
  check_launch("payload_compact");
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "gfx950 HIP kernels for the bitmap index";
  m.attr("QUERYPROG_BYTES") = int(sizeof(pk::QueryProg));
  m.attr("VIEWDEV_BYTES") = int(sizeof(pk::ViewDev));
  m.attr("MAXLEAF") = pk::MAXLEAF;
  m.attr("MAXPROG") = pk::MAXPROG;
  m.def("expr_count", &expr_count, "batched boolean-expression count over all local shards",
        py::arg("progs"), py::arg("views"), py::arg("S"), py::arg("out"), py::arg("per_key"), py::arg("mode") = 0,
        py::arg("per_shard") = py::none());
  m.def("expr_materialize", &expr_materialize, "write result containers for a batch of expressions");
#ifdef PK_KBENCH
  m.def("shadow_build", &shadow_build, "dense bitmap shadows of hot rows for the pair kernels");
  m.attr("KBENCH") = true;
#else
  m.attr("KBENCH") = false;
#endif
  m.def("partial_sum_scatter", &partial_sum_scatter, "out[ti[q]] += column sums of int32[U][n] partials");
  m.def("and2_count", &and2_count, "Count(Intersect(a,b)) batch via key-major pair kernels", py::arg("progs"),
        py::arg("views"), py::arg("S"), py::arg("pairs"), py::arg("partial"), py::arg("cq") = 0,
        py::arg("variant") = 1);
  m.def("bsi_range", &bsi_range, "BSI predicate -> bitmap container per (shard, key)");
  m.def("bsi_range_count", &bsi_range_count, "Count(Row(v <op> x)): fused BSI predicate + count");
  m.def("bsi_minmax", &bsi_minmax, "BSI min/max descents per (shard, key); which: 0 both, 1 Min, 2 Max",
        py::arg("progs"), py::arg("views"), py::arg("S"), py::arg("bsi_args"), py::arg("out"), py::arg("which") = 0);
  m.def("leaf_src", &leaf_src, "src containers of plain rows straight from the arena (TopN srcs)");
  m.def("row_counts", &row_counts, "row counts of (shard, dense row) entries (device rank caches)");
  m.def("topn_cache_counts", &topn_cache_counts, "cache-only TopN: [candidate x shard] row counts");
  m.def("topn_cache_batch", &topn_cache_batch, "cache-only TopN batch: membership, totals, per-query top-n");
  m.def("mesh_cache_issue", &mesh_cache_issue, "mesh cache-only TopN share: params, partial buffer (pre all-reduce)");
  m.def("mesh_cache_finish", &mesh_cache_finish, "mesh cache-only TopN: select, D2H, decode (post all-reduce)");
  py::class_<CacheTopN>(m, "CacheTopN")
      .def(py::init<torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, int64_t, torch::Tensor>())
      .def("run", &CacheTopN::run, "cache-only TopN batch end to end: (ids, counts, offsets) or None")
      .def_property_readonly("U", &CacheTopN::U)
      .def_property_readonly("stride", &CacheTopN::stride);
  m.def("upload_i32", &upload_i32, "small host int32 array -> device through a pinned ring (current stream)");
  m.def("topn_cache_partial", &topn_cache_partial, "mesh cache-only TopN: one rank's membership + partial totals");
  m.def("topn_cache_select32", &topn_cache_select32, "mesh cache-only TopN: per-query top-n of the reduced buffer");
  m.def("row_counts_sum", &row_counts_sum, "ids= re-count without src: per id the sum of shard row counts >= threshold");
  m.def("keymask_build", &keymask_build, "key-presence mask of every (shard, row) of a view");
  m.def("topn_hot_meta", &topn_hot_meta, "key-j container of every hot cache rank of the TopN index");
  m.def("topn_index", &topn_index, "build pass of the device TopN slot index (count or fill)");
  m.def("bsi_minmax_fold", &bsi_minmax_fold, "fold BSI min/max descents into one (value, count, found)");
  m.def("topn_src", &topn_src, "src-filtered TopN over the slot index: mode 1 heap walk, mode 2/3 ids= re-count (rebuilt / kept histograms)");
  m.def("bitgemm", &bitgemm, "row-pair intersection count matrix of dense bit rows (mode 1 MFMA i8, 0 VALU)");
  m.def("expr_dense", &expr_dense, "evaluate expressions into dense one-row views (bitmap per shard/key)");
  m.def("shift_dense", &shift_dense, "Shift a dense view by n columns per shard (main + next-shard spill)",
        py::arg("src"), py::arg("S"), py::arg("n"), py::arg("main_out"), py::arg("main_meta"), py::arg("spill_out"),
        py::arg("spill_meta"), py::arg("M") = 1, py::arg("row_words") = 16384);
  m.def("rows_list", &rows_list, "flag dense rows with non-empty containers (optionally holding one column)");
  m.def("container_merge", &container_merge, "device write path: old container + delta -> bitmap + cardinality");
  m.def("payload_compact", &payload_compact, "copy live containers into a compacted payload buffer");
  m.def("container_emit", &container_emit, "device write path: bitmap -> final run/array/bitmap container (Optimize rule) + metadata");
  m.def("densify", &densify, "dense bit rows of an arena over a shard range");
  m.def("bsi_sum", &bsi_sum, "bit-sliced integer sum with optional filter program", py::arg("progs"),
        py::arg("views"), py::arg("S"), py::arg("bsi_args"), py::arg("out_sum"), py::arg("out_cnt"),
        py::arg("fmode") = 2);
}
