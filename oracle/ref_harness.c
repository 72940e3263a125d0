/*
 * oracle/ref_harness.c -- TEST / BASELINE INFRASTRUCTURE ONLY.
 *
 * Linked (by oracle/Makefile) together with the reference's own crc.c, compiled
 * straight from /root/reference/crc.c, into oracle/_ref/libref_crc.so.  This file
 * is ours; it contains no reference source.  It lets tests and bench.py's
 * cpu_baseline leg call the *real* reference rpc_crc32() (crc.c:4-9, which calls
 * system zlib crc32 exactly as crc.c:6-7 does) over a batch, on N host threads.
 *
 * Never used by the product library.
 */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <stdbool.h>
#include <time.h>

/* From the reference crc.h:8,11 (linked from /root/reference/crc.c). */
uint32_t rpc_crc32(const void *data, size_t len);
bool rpc_crc32_verify(const void *data, size_t len, uint32_t expected_crc);

uint32_t ref_rpc_crc32(const void *data, size_t len) { return rpc_crc32(data, len); }
int ref_rpc_crc32_verify(const void *data, size_t len, uint32_t e) { return rpc_crc32_verify(data, len, e) ? 1 : 0; }

typedef struct {
    const uint8_t *base;
    const uint64_t *offsets; /* NULL -> uniform: i*stride */
    const uint32_t *lengths; /* NULL -> uniform: len */
    uint64_t stride;
    uint32_t len;
    uint64_t lo, hi;
    uint32_t *out;
    int reps;
} ref_job_t;

static void *ref_worker(void *arg)
{
    ref_job_t *j = (ref_job_t *)arg;
    for (int r = 0; r < j->reps; r++) {
        for (uint64_t i = j->lo; i < j->hi; i++) {
            uint64_t off = j->offsets ? j->offsets[i] : i * j->stride;
            uint32_t len = j->lengths ? j->lengths[i] : j->len;
            j->out[i] = rpc_crc32(j->base + off, len);
        }
    }
    return NULL;
}

/* Runs the batch `reps` times on `threads` threads (static partition) and
 * returns the wall time in seconds.  out[] holds the CRCs of the last rep. */
double ref_crc32_batch_timed(const uint8_t *base, const uint64_t *offsets,
                             const uint32_t *lengths, uint64_t n, uint32_t len,
                             uint64_t stride, uint32_t *out, int threads, int reps)
{
    if (threads < 1)
        threads = 1;
    if (threads > 256)
        threads = 256;
    pthread_t tid[256];
    ref_job_t jobs[256];
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < threads; t++) {
        jobs[t].base = base;
        jobs[t].offsets = offsets;
        jobs[t].lengths = lengths;
        jobs[t].stride = stride;
        jobs[t].len = len;
        jobs[t].lo = n * (uint64_t)t / (uint64_t)threads;
        jobs[t].hi = n * (uint64_t)(t + 1) / (uint64_t)threads;
        jobs[t].out = out;
        jobs[t].reps = reps;
        if (t > 0)
            pthread_create(&tid[t], NULL, ref_worker, &jobs[t]);
    }
    ref_worker(&jobs[0]);
    for (int t = 1; t < threads; t++)
        pthread_join(tid[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
