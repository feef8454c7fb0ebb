/*
 * vs_client.c — a plain C host of the engine's C-ABI (include/vsearch.h),
 * linked with -lvsearch: what rag/vector-service's cgo binding does, minus
 * Go. create -> upsert -> search -> results to a file, which the test checks
 * against the oracle (tests/test_c_client_gpu.py).
 *
 *   vs_client SHARDS DTYPE corpus.f32 N DIM queries.f32 NQ K out.bin
 *
 * SHARDS = 0: vs_open on device 0; SHARDS >= 1: vs_open_multi with that many
 * shards on device 0. out.bin: NQ*K f32 scores, NQ*K u64 rows, NQ u32 counts.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "vsearch.h"

static void* slurp(const char* path, size_t want) {
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  void* p = malloc(want ? want : 1);
  size_t got = p ? fread(p, 1, want, f) : 0;
  fclose(f);
  if (got != want) {
    free(p);
    return NULL;
  }
  return p;
}

#define CHECK(call)                                                        \
  do {                                                                     \
    int rc_ = (call);                                                      \
    if (rc_ != VS_OK) {                                                    \
      fprintf(stderr, "%s failed: %d %s\n", #call, rc_, vs_last_error()); \
      return 2;                                                            \
    }                                                                      \
  } while (0)

int main(int argc, char** argv) {
  if (argc != 10) {
    fprintf(stderr, "usage: %s SHARDS DTYPE corpus N DIM queries NQ K out\n", argv[0]);
    return 1;
  }
  const int shards = atoi(argv[1]), dtype = atoi(argv[2]);
  const uint64_t n = strtoull(argv[4], NULL, 10);
  const uint32_t dim = (uint32_t)atoi(argv[5]), nq = (uint32_t)atoi(argv[7]),
                 k = (uint32_t)atoi(argv[8]);
  float* X = (float*)slurp(argv[3], n * dim * sizeof(float));
  float* Q = (float*)slurp(argv[6], (size_t)nq * dim * sizeof(float));
  if (!X || !Q) {
    fprintf(stderr, "cannot read inputs\n");
    return 1;
  }
  vs_engine* eng = NULL;
  if (shards == 0) {
    vs_config cfg = {0, 0};
    CHECK(vs_open(&cfg, &eng));
  } else {
    int32_t* devs = (int32_t*)calloc((size_t)shards, sizeof(int32_t));
    vs_config_multi cfg = {devs, (uint32_t)shards, 0};
    CHECK(vs_open_multi(&cfg, &eng));
    free(devs);
  }
  uint32_t s = 0, d = 0;
  CHECK(vs_engine_layout(eng, &s, &d));
  if (s != (uint32_t)(shards ? shards : 1) || d != 1) return 3;
  /* initializeCollections: Get -> NotFound -> Create (main.go:91-112) */
  if (vs_collection_info(eng, "regulatory_docs", NULL, NULL, NULL, NULL) != VS_ERR_NOT_FOUND)
    return 4;
  CHECK(vs_collection_create(eng, "regulatory_docs", dim, VS_METRIC_COSINE, dtype, 0, 0));
  uint64_t* rows = (uint64_t*)malloc(n * sizeof(uint64_t));
  for (uint64_t i = 0; i < n; ++i) rows[i] = i;
  /* two upserts, the second overwrites row 3 with row 3's vector again */
  CHECK(vs_upsert(eng, "regulatory_docs", n, dim, rows, X));
  CHECK(vs_upsert(eng, "regulatory_docs", 1, dim, rows + 3, X + 3 * (size_t)dim));
  uint64_t have = 0;
  CHECK(vs_collection_info(eng, "regulatory_docs", NULL, &have, NULL, NULL));
  if (have != n) return 5;
  /* a wrong-size query is a dimension error, not a crash */
  if (vs_search(eng, "regulatory_docs", Q, 1, dim - 1, k, NULL, NULL, NULL) != VS_ERR_DIM_MISMATCH)
    return 6;
  float* scores = (float*)calloc((size_t)nq * k, sizeof(float));
  uint64_t* out_rows = (uint64_t*)calloc((size_t)nq * k, sizeof(uint64_t));
  uint32_t* counts = (uint32_t*)calloc(nq, sizeof(uint32_t));
  CHECK(vs_search(eng, "regulatory_docs", Q, nq, dim, k, scores, out_rows, counts));
  char health[4096];
  CHECK(vs_health(eng, health, sizeof(health)));
  if (!strstr(health, "\"healthy\"")) return 7;
  FILE* f = fopen(argv[9], "wb");
  if (!f) return 8;
  fwrite(scores, sizeof(float), (size_t)nq * k, f);
  fwrite(out_rows, sizeof(uint64_t), (size_t)nq * k, f);
  fwrite(counts, sizeof(uint32_t), nq, f);
  fclose(f);
  vs_close(eng);
  free(X), free(Q), free(rows), free(scores), free(out_rows), free(counts);
  printf("ok %s\n", health);
  return 0;
}
