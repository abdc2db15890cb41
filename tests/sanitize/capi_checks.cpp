// Host-side argument checks of the C-ABI (include/hrec.h) under
// AddressSanitizer + UndefinedBehaviorSanitizer ("host ASan/UBSan
// on C-ABI glue"). Built by tests/test_sanitizers.py from the library
// sources with the sanitizers on the host side only (each -fsanitize= after
// -Xarch_host; the gfx950 code is built as usual and never launched), so it
// needs no GPU: every call below must be rejected by its
// HREC_REQUIRE checks (HREC_E_INVALID + a message) before any HIP call, and
// the workspace-size queries must stay free of overflow / UB over a sweep of
// shapes. The thread-local hrec_last_error is exercised from two threads.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <thread>

#include "../../include/hrec.h"

static int failures = 0;

static void expect_invalid(int rc, const char* what) {
  const char* msg = hrec_last_error();
  if (rc != HREC_E_INVALID || msg == nullptr || msg[0] == '\0') {
    fprintf(stderr, "FAIL %s: rc=%d msg=%s\n", what, rc, msg ? msg : "(null)");
    ++failures;
  }
}

#define INVALID(call) expect_invalid((call), #call)

int main() {
  if (hrec_abi_version() != HREC_ABI_VERSION) {
    fprintf(stderr, "FAIL abi version\n");
    return 1;
  }
  // synth / scan / ingest
  INVALID(hrec_synth_row_counts(1, 1, 0, -1, 10, 0, nullptr, nullptr));
  INVALID(hrec_synth_fill(1, 2, 1, 0, -1, 10, 0, 19, nullptr, nullptr, nullptr, nullptr));
  INVALID(hrec_exclusive_scan_i64(nullptr, -1, nullptr, nullptr, 0, nullptr));
  INVALID(hrec_minmax_i64(nullptr, 0, nullptr, nullptr, 0, nullptr));
  INVALID(hrec_encode_ids(nullptr, -1, 0, 0, nullptr, nullptr, nullptr, nullptr, 0, nullptr));
  INVALID(hrec_coo_to_csr(nullptr, nullptr, nullptr, -1, 4, nullptr, nullptr, nullptr, nullptr, 0, nullptr));
  INVALID(hrec_remap_i32(nullptr, -1, nullptr, 0, nullptr));
  INVALID(hrec_rows_descending_pairs(nullptr, 4, nullptr, nullptr));
  INVALID(hrec_coo_to_csr_sorted(nullptr, nullptr, nullptr, -1, 4, nullptr, nullptr, nullptr, nullptr));
  // ALS
  INVALID(hrec_als_init_factors(1, 0, 4, 65, 64, nullptr, nullptr));
  INVALID(hrec_als_half_sweep(nullptr, nullptr, nullptr, 4, nullptr, 4, 8, 48, 0.1, 0, nullptr, nullptr));
  INVALID(hrec_als_half_sweep(nullptr, nullptr, nullptr, 4, nullptr, 4, 8, 16, 0.1, 7, nullptr, nullptr));
  INVALID(hrec_als_half_sweep_src64(nullptr, nullptr, nullptr, 4, nullptr, 4, 8, 32, 0.1, nullptr, nullptr));
  INVALID(hrec_f32_to_f64(nullptr, -1, nullptr, nullptr));
  INVALID(hrec_transpose_f32(nullptr, -1, 4, nullptr, 4, nullptr));
  INVALID(hrec_als_score(nullptr, nullptr, 1, nullptr, 4, nullptr, 4, 8, 48, nullptr, nullptr));
  INVALID(hrec_als_score_topk(nullptr, nullptr, 1, nullptr, 4, 4, 8, 48, 5, nullptr, nullptr, nullptr, nullptr, 0,
                              nullptr));
  // top-k / fusion
  INVALID(hrec_topk_f32(nullptr, -1, 4, 4, 1, nullptr, nullptr, nullptr, 0, nullptr));
  INVALID(hrec_topk_f64(nullptr, 1, -4, 4, 1, nullptr, nullptr, nullptr, 0, nullptr));
  INVALID(hrec_fuse_topk(nullptr, nullptr, 1, -1, 1, 5, nullptr, nullptr, nullptr, nullptr, nullptr, 0, nullptr));
  INVALID(hrec_rows_minmax_f32(nullptr, -1, 4, 4, nullptr, nullptr));
  INVALID(hrec_fuse_rows_topk(nullptr, nullptr, 1, 0, 0, nullptr, nullptr, 1, 5, 0, nullptr, nullptr, nullptr, 0,
                              nullptr));
  INVALID(hrec_topk_f64_keyed(nullptr, nullptr, 1, 4, 0, nullptr, nullptr, nullptr, 0, nullptr));
  INVALID(hrec_cosine_sim(nullptr, -1, 4, nullptr, 1, nullptr, nullptr));
  // two-tower
  hrec_tt_params p;
  memset(&p, 0, sizeof(p));
  p.d = 0;
  INVALID(hrec_tt_item_forward(&p, nullptr, nullptr, nullptr, nullptr, 4, nullptr, nullptr));
  INVALID(hrec_tt_user_forward(&p, nullptr, 4, nullptr, nullptr));
  INVALID(hrec_tt_score(nullptr, -1, nullptr, 4, 8, nullptr, nullptr));
  INVALID(hrec_tt_pair_score(nullptr, nullptr, -1, 8, nullptr, nullptr));
  INVALID(hrec_tt_forward_backward(&p, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 4, nullptr, nullptr,
                                   nullptr, nullptr, nullptr, nullptr, 0, nullptr));
  INVALID(hrec_adam_dense(nullptr, nullptr, nullptr, nullptr, -1, 0.1f, 0.9f, 0.999f, 1e-7f, nullptr));
  INVALID(hrec_adam_sparse(nullptr, nullptr, nullptr, -1, 8, nullptr, nullptr, 4, nullptr, nullptr, 0.1f, 0.9f, 0.1f,
                           0.999f, 0.001f, 1e-7f, nullptr));
  INVALID(hrec_adam_sparse_tables(nullptr, HREC_MAX_SPARSE_TABLES + 1, 0.1f, 0.9f, 0.1f, 0.999f, 0.001f, 1e-7f,
                                  nullptr));
  INVALID(hrec_adam_sparse_tables_phase(nullptr, 1, 9, 0.1f, 0.9f, 0.1f, 0.999f, 0.001f, 1e-7f, nullptr));
  // matrix-core scoring / hybrid
  INVALID(hrec_f32_to_bf16(nullptr, -1, nullptr, nullptr));
  INVALID(hrec_dot_scores(nullptr, 1, nullptr, 4, 48, 0, nullptr, 4, nullptr));
  INVALID(hrec_dot_topk(nullptr, 1, nullptr, 4, 64, 2, 5, nullptr, 0, nullptr, nullptr, nullptr, nullptr, 0, nullptr));
  INVALID(hrec_dot_filter(nullptr, 1, nullptr, 4, 256, 0, nullptr, 1, 0, 8, nullptr, nullptr, nullptr, nullptr));
  INVALID(hrec_dot_filter(nullptr, 1, nullptr, 100, 64, 1, nullptr, 2, 32, -8, nullptr, nullptr, nullptr, nullptr));
  INVALID(hrec_hybrid_scores(nullptr, 64, nullptr, -1, 64, nullptr, 64, 64, 4, nullptr, nullptr, 10, 64, nullptr,
                             nullptr, 10, nullptr, nullptr, nullptr, 0, nullptr));
  INVALID(hrec_hybrid_prune_minmax(nullptr, 64, nullptr, 4, 64, nullptr, 64, 64, 4, nullptr, nullptr, 10, 96,
                                   nullptr, nullptr, nullptr, 0, nullptr));
  INVALID(hrec_hybrid_prune_topk(nullptr, 64, nullptr, 4, 64, nullptr, 64, 64, 4, nullptr, nullptr, 10, 64, nullptr,
                                 nullptr, 1, 9, 0, nullptr, nullptr, nullptr, 0, nullptr));
  INVALID(hrec_hybrid_prune_fallback_taken(nullptr, 1, 1, 64, 5, nullptr, nullptr));
  INVALID(hrec_hybrid_prune_local(nullptr, 64, nullptr, 4, 64, nullptr, 64, 64, 4, nullptr, nullptr, 10, 64, 0, 9, 0,
                                  nullptr, nullptr, nullptr, nullptr, nullptr, 0, nullptr));
  INVALID(hrec_hybrid_prune_survivors(nullptr, 1, 1, 64, 5, nullptr, nullptr));

  // RCCL exchange steps (argument checks only: no communicator exists here)
  INVALID(hrec_comm_get_unique_id(nullptr));
  INVALID(hrec_comm_init(0, 1, nullptr, nullptr));
  INVALID(hrec_allgather(nullptr, nullptr, nullptr, 4, 0, nullptr));
  INVALID(hrec_allreduce_minmax(nullptr, nullptr, 1, 4, nullptr));

  // workspace-size queries over a sweep of shapes (UBSan: no signed overflow)
  size_t acc = 0;
  const int64_t ns[] = {0, 1, 17, 1000, 100003, 50000000};
  const int bs[] = {0, 1, 256, 1024, 65535};
  const int ks[] = {1, 5, 8, 64, 1024};
  for (int64_t n : ns)
    for (int b : bs)
      for (int k : ks) {
        acc += hrec_als_score_topk_workspace_bytes(b, n, k);
        acc += hrec_topk_workspace_bytes(b, n, k, 1) + hrec_topk_workspace_bytes(b, n, k, 0);
        acc += hrec_fuse_workspace_bytes(n, k) + hrec_fuse_rows_workspace_bytes(b, n, k);
        acc += hrec_dot_topk_workspace_bytes(b, n, k);
        acc += hrec_hybrid_scores_workspace_bytes(b, n);
        if (k <= 8) acc += hrec_hybrid_prune_workspace_bytes(b, n, 256, k);
      }
  for (int64_t n : ns) {
    acc += hrec_scan_workspace_bytes(n) + hrec_minmax_i64_workspace_bytes(n) + hrec_encode_ids_workspace_bytes(n);
    acc += hrec_coo_to_csr_workspace_bytes(n, n / 3 + 1) + hrec_tt_train_workspace_bytes(64, n);
  }
  acc += hrec_tt_grad_len(256);
  if (acc == 0) ++failures;

  // hrec_last_error is thread-local: a failure on another thread leaves ours alone
  INVALID(hrec_f32_to_f64(nullptr, -1, nullptr, nullptr));
  char mine[256];
  snprintf(mine, sizeof(mine), "%s", hrec_last_error());
  std::thread t([] { hrec_topk_f32(nullptr, -1, 4, 4, 1, nullptr, nullptr, nullptr, 0, nullptr); });
  t.join();
  if (strcmp(mine, hrec_last_error()) != 0) {
    fprintf(stderr, "FAIL last_error is not thread-local\n");
    ++failures;
  }
  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  printf("capi_checks OK\n");
  return 0;
}
