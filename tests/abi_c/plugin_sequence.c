/*
 * plugin_sequence.c -- the cgo grep plugin's call sequence against libdgrep.so,
 * written in C against include/dgrep.h (what INTEGRATION.md's Go binding does):
 *
 *   dgrep_compile -> dgrep_open -> dgrep_load_dfa -> dgrep_scan ->
 *   dgrep_result_free -> ... -> dgrep_close
 *
 * plus the error paths a plugin relies on (dgrep_last_error after a malformed
 * blob, DGREP_E_NO_DFA before a load) and a scan issued from a second pthread
 * on the same context (a Go goroutine may run on any OS thread,
 * main/worker_launch.go:16-18 -> map_reduce/worker.go:126-145).
 *
 * Usage: plugin_sequence <pattern-file> <split-file> <out-file>
 * Writes the records of the main-thread scan, the pthread scan and a second
 * context's scan on the same device, as "line_no start len" lines, each block preceded by "# <count>". Exit 0 on
 * success; tests/test_abi_c.py compares the output with the oracle.
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dgrep.h"

static unsigned char* slurp(const char* path, size_t* n) {
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  long len = ftell(f);
  fseek(f, 0, SEEK_SET);
  unsigned char* buf = malloc(len > 0 ? (size_t)len : 1);
  if (len > 0 && fread(buf, 1, (size_t)len, f) != (size_t)len) {
    fclose(f);
    free(buf);
    return NULL;
  }
  fclose(f);
  *n = (size_t)len;
  return buf;
}

#define CHECK(cond, ...)                    \
  do {                                      \
    if (!(cond)) {                          \
      fprintf(stderr, "FAIL: " __VA_ARGS__); \
      fprintf(stderr, "\n");                \
      exit(1);                              \
    }                                       \
  } while (0)

struct job {
  dgrep_ctx* ctx;
  const unsigned char* data;
  size_t n;
  dgrep_result res;
  int rc;
};

static void* scan_thread(void* p) {
  struct job* j = p;
  j->rc = dgrep_scan(j->ctx, j->data, j->n, &j->res);
  return NULL;
}

static void dump(FILE* out, const dgrep_result* r) {
  fprintf(out, "# %llu\n", (unsigned long long)r->count);
  for (uint64_t i = 0; i < r->count; ++i)
    fprintf(out, "%llu %llu %llu\n", (unsigned long long)r->line_no[i], (unsigned long long)r->start[i],
            (unsigned long long)r->len[i]);
}

int main(int argc, char** argv) {
  CHECK(argc == 4, "usage: plugin_sequence <pattern-file> <split-file> <out-file>");
  size_t plen = 0, n = 0;
  unsigned char* pattern = slurp(argv[1], &plen);
  unsigned char* data = slurp(argv[2], &n);
  CHECK(pattern && data, "cannot read inputs");

  /* regexp.Compile once per pattern (grep.go:21 compiles per line) */
  void* blob = NULL;
  size_t blen = 0;
  char err[256] = {0};
  int rc = dgrep_compile((const char*)pattern, plen, &blob, &blen, err, sizeof err);
  CHECK(rc == DGREP_OK, "dgrep_compile rc=%d: %s", rc, err);
  dgrep_blob_info info;
  CHECK(dgrep_blob_info_get(blob, blen, &info) == DGREP_OK, "blob info");

  /* the worker's device: DGREP_DEVICE, else worker id % device count */
  int dev = -1;
  rc = dgrep_pick_device(-1, &dev);
  CHECK(rc == DGREP_OK, "dgrep_pick_device rc=%d (DGREP_DEVICE=%s)", rc,
        getenv("DGREP_DEVICE") ? getenv("DGREP_DEVICE") : "unset");
  dgrep_ctx* ctx = NULL;
  rc = dgrep_open(dev, &ctx);
  CHECK(rc == DGREP_OK, "dgrep_open rc=%d: %s", rc, ctx ? dgrep_last_error(ctx) : "");
  /* a second context on the same device (one per stream; no shared state) */
  dgrep_ctx* ctx2 = NULL;
  rc = dgrep_open(dev, &ctx2);
  CHECK(rc == DGREP_OK, "second dgrep_open rc=%d", rc);

  /* a scan before any pattern: DGREP_E_NO_DFA with a message */
  dgrep_result r0;
  rc = dgrep_scan(ctx, data, n, &r0);
  CHECK(rc == DGREP_E_NO_DFA && strlen(dgrep_last_error(ctx)) > 0, "scan before load rc=%d", rc);

  /* a malformed blob: DGREP_E_INVALID, dgrep_last_error says why */
  unsigned char junk[64];
  memset(junk, 0xab, sizeof junk);
  rc = dgrep_load_dfa(ctx, junk, sizeof junk);
  CHECK(rc == DGREP_E_INVALID && strlen(dgrep_last_error(ctx)) > 0, "malformed blob rc=%d", rc);

  rc = dgrep_load_dfa(ctx, blob, blen);
  CHECK(rc == DGREP_OK, "dgrep_load_dfa rc=%d: %s", rc, dgrep_last_error(ctx));
  rc = dgrep_load_dfa(ctx2, blob, blen);
  CHECK(rc == DGREP_OK, "second dgrep_load_dfa rc=%d: %s", rc, dgrep_last_error(ctx2));
  dgrep_blob_free(blob);

  FILE* out = fopen(argv[3], "w");
  CHECK(out, "cannot write %s", argv[3]);

  /* Map on the thread that opened the context */
  dgrep_result r;
  rc = dgrep_scan(ctx, data, n, &r);
  CHECK(rc == DGREP_OK, "dgrep_scan rc=%d: %s", rc, dgrep_last_error(ctx));
  dump(out, &r);
  dgrep_result_free(&r);
  CHECK(r.count == 0 && r.line_no == NULL, "dgrep_result_free clears the result");

  /* the same context from another OS thread */
  struct job j = {ctx, data, n, {0, NULL, NULL, NULL}, -1};
  pthread_t th;
  CHECK(pthread_create(&th, NULL, scan_thread, &j) == 0, "pthread_create");
  pthread_join(th, NULL);
  CHECK(j.rc == DGREP_OK, "pthread dgrep_scan rc=%d: %s", j.rc, dgrep_last_error(ctx));
  dump(out, &j.res);
  dgrep_result_free(&j.res);

  /* the second context scans the same split independently */
  dgrep_result r2;
  rc = dgrep_scan(ctx2, data, n, &r2);
  CHECK(rc == DGREP_OK, "second context dgrep_scan rc=%d: %s", rc, dgrep_last_error(ctx2));
  dump(out, &r2);
  dgrep_result_free(&r2);
  dgrep_close(ctx2);

  fclose(out);
  dgrep_close(ctx);
  free(pattern);
  free(data);
  printf("plugin sequence OK (%u DFA states)\n", info.nstates);
  return 0;
}
