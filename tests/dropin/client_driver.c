/*
 * tests/dropin/client_driver.c -- TEST INFRASTRUCTURE: a driver `main` for the
 * reference's own client library (client/rpc_async.c, conn_pool.c, pending.c,
 * epoll_api.c, rpc_codec.c, gen/rpc_client_gen.c, third_party/cJSON.c),
 * compiled in place by `make -C oracle dropin` and linked against librpccrc.so
 * INSTEAD OF crc.c.  The reference's own main (rpc_client_main.c) idles under
 * TEST_IDLE (rpc_client_main.c:113), so this driver replaces it with the same
 * shape of work: THREAD_COUNT = 10 user threads (rpc_client_main.c:17) calling
 * the generated stubs concurrently.  Every request is stamped by rpc_crc32 at
 * rpc_async.c:525 and every response verified by rpc_crc32_verify at
 * rpc_async.c:219 -- both now on the GPU.
 *
 *   client_rpccrc stress <port> <threads> <calls>
 *       threads x calls rounds of add_i32 / echo_i64 / strlen_s against a server;
 *       prints {"success": S, "failure": F}
 *   client_rpccrc raw <port> <json>
 *       one rpc_call_async_blocking; prints {"status": <rpc_error_code>}
 *       (RPC_CRC_ERR = 5 when the response CRC does not verify, rpc_types.h:27)
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rpc_async.h"
#include "rpc_client_gen.h"

static int g_calls = 10;

typedef struct {
  int id;
  int success;
  int failure;
} worker_t;

static void *worker(void *arg) {
  worker_t *w = (worker_t *)arg;
  for (int i = 0; i < g_calls; ++i) {
    const int32_t a = 1000 * w->id + i + 1, b = 7 * i + 3;
    const int64_t x = 1234567890123LL + 17 * w->id + i;
    char s[64];
    snprintf(s, sizeof s, "thread-%d-call-%d", w->id, i);
    const int ok = add_i32(a, b) == a + b && echo_i64(x) == x && strlen_s(s) == (int32_t)strlen(s);
    if (ok)
      w->success++;
    else
      w->failure++;
  }
  return NULL;
}

int main(int argc, char **argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s stress <port> <threads> <calls> | raw <port> <json>\n", argv[0]);
    return 2;
  }
  const int port = atoi(argv[2]);
  if (rpc_async_init("127.0.0.1", port, 20, 10000) != 0) {
    fprintf(stderr, "rpc_async_init failed\n");
    return 1;
  }
  int rc = 0;
  if (strcmp(argv[1], "stress") == 0 && argc >= 5) {
    const int nthreads = atoi(argv[3]);
    g_calls = atoi(argv[4]);
    pthread_t th[64];
    worker_t ws[64];
    int n = nthreads > 64 ? 64 : nthreads;
    for (int i = 0; i < n; ++i) {
      ws[i].id = i;
      ws[i].success = ws[i].failure = 0;
      pthread_create(&th[i], NULL, worker, &ws[i]);
    }
    int succ = 0, fail = 0;
    for (int i = 0; i < n; ++i) {
      pthread_join(th[i], NULL);
      succ += ws[i].success;
      fail += ws[i].failure;
    }
    printf("{\"success\": %d, \"failure\": %d}\n", succ, fail);
    rc = fail ? 1 : 0;
  } else if (strcmp(argv[1], "raw") == 0 && argc >= 4) {
    char *body = NULL;
    size_t len = 0;
    rpc_error_code status = RPC_OK;
    (void)rpc_call_async_blocking(argv[3], rpc_async_next_id(), &body, &len, &status);
    printf("{\"status\": %d}\n", (int)status);
    free(body);
  } else {
    fprintf(stderr, "bad arguments\n");
    rc = 2;
  }
  fflush(stdout);
  rpc_async_shutdown();
  return rc;
}
