// tools/scalar_bench.c -- MEASUREMENT ONLY: per-call latency of the drop-in
// rpc_crc32 (crc.h:8) as the reference's callers use it -- one body per call
// from a user thread (client stamp rpc_async.c:525, up to 10 user threads,
// rpc_client_main.c:17; server verify rpc_server_main.c:227) -- through
// librpccrc (one GPU kernel per call) next to the reference's own crc.c
// (oracle/_ref/libref_crc.so, dlopen'ed; system zlib) on the same host.
//
// usage: scalar_bench [ref_lib]     prints one JSON object
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "rpccrc.h"

typedef uint32_t (*crc_fn)(const void *, size_t);

static double now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

typedef struct {
  crc_fn fn;
  const uint8_t *body;
  size_t len;
  long calls;
  uint32_t want;
  long bad;
  double secs;
} job_t;

static void *run(void *arg) {
  job_t *j = (job_t *)arg;
  const double t0 = now();
  for (long i = 0; i < j->calls; ++i) j->bad += j->fn(j->body, j->len) != j->want;
  j->secs = now() - t0;
  return NULL;
}

// Mean microseconds per call seen by each of `threads` threads calling
// concurrently (max over threads), and the aggregate calls per second.
static void measure(crc_fn fn, const uint8_t *body, size_t len, int threads, long calls, uint32_t want,
                    double *us_per_call, double *calls_per_s, long *bad) {
  pthread_t th[64];
  job_t jobs[64];
  for (int t = 0; t < threads; ++t) {
    jobs[t] = (job_t){fn, body, len, calls, want, 0, 0};
    pthread_create(&th[t], NULL, run, &jobs[t]);
  }
  double worst = 0;
  *bad = 0;
  for (int t = 0; t < threads; ++t) {
    pthread_join(th[t], NULL);
    if (jobs[t].secs > worst) worst = jobs[t].secs;
    *bad += jobs[t].bad;
  }
  *us_per_call = worst / calls * 1e6;
  *calls_per_s = threads * calls / worst;
}

int main(int argc, char **argv) {
  crc_fn ref = NULL;
  if (argc > 1) {
    void *h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
    ref = h ? (crc_fn)dlsym(h, "ref_rpc_crc32") : NULL;
  }
  // Bodies: the captured request (68 B), a 12-byte body and 1 KiB
  // (MAX_BODY_LEN, rpc.h:17) of JSON-like text.
  static uint8_t buf[1024];
  const char *req = "{\"jsonrpc\":\"2.0\",\"method\":\"add_i32\",\"params\":{\"a\":10,\"b\":20},\"id\":1}";
  for (int i = 0; i < 1024; ++i) buf[i] = (uint8_t)(32 + (i * 37 + 11) % 95);
  const size_t sizes[3] = {12, 68, 1024};
  // Warm-up outside the timed loops: 10 concurrent callers make the library
  // create its 10 pooled scalar contexts (stream + pinned staging each), so
  // every timed row is steady state (the first 10-thread row
  // used to include that growth).
  {
    double us, cps;
    long bad;
    const uint32_t w = rpc_crc32(buf, 64);
    measure((crc_fn)rpc_crc32, buf, 64, 10, 200, w, &us, &cps, &bad);
  }
  printf("{\"unit\": \"us_per_call\", \"rows\": [");
  int first = 1, fail = 0;
  for (int si = 0; si < 3; ++si) {
    const size_t len = sizes[si];
    uint8_t body[1024];
    memcpy(body, buf, len);
    if (len == 68) memcpy(body, req, 68);
    const uint32_t want = rpc_crc32(body, len); // warms the device context
    if (ref && ref(body, len) != want) fail = 1;
    // SCALAR_BENCH_THREADS="1,2,4,..." replaces the thread counts (a probe of
    // how the drop-in scales; the default rows are the reference's 1 and 10).
    int tcounts[16] = {1, 10}, nt = 2;
    if (getenv("SCALAR_BENCH_THREADS")) {
      nt = 0;
      for (char *p = getenv("SCALAR_BENCH_THREADS"); *p && nt < 16;) {
        tcounts[nt++] = (int)strtol(p, &p, 10);
        if (*p == ',') ++p;
        else break;
      }
    }
    for (int ti = 0; ti < nt; ++ti) {
      const int th = tcounts[ti];
      double us, cps, rus = -1, rcps = -1;
      long bad, rbad = 0;
      measure((crc_fn)rpc_crc32, body, len, th, 2000, want, &us, &cps, &bad);
      if (ref) measure(ref, body, len, th, 2000000 / (long)(len < 64 ? 64 : len) * 16, want, &rus, &rcps, &rbad);
      fail |= bad != 0 || rbad != 0;
      printf("%s{\"bytes\": %zu, \"threads\": %d, \"gpu_us\": %.3f, \"gpu_calls_per_s\": %.0f, "
             "\"ref_us\": %.4f, \"ref_calls_per_s\": %.0f}",
             first ? "" : ", ", len, th, us, cps, rus, rcps);
      first = 0;
    }
  }
  printf("], \"ok\": %s}\n", fail ? "false" : "true");
  return fail ? 3 : 0;
}
