/*
 * coalesce_bench.c -- latency and throughput of the single-message path
 * (net2_hashctx_hashiov, i.e. net2_hashctx_hashbuf at types/signature.n2t:92,
 * 147) under concurrency: T host threads, as the reference's threadpool
 * workers (include/ilias/net2/threadpool.h:33-34), each hashing one message
 * per call in a loop for a fixed time.  Prints one JSON line per thread
 * count: median / p99 latency per call and the aggregate messages/s.
 *
 *   coalesce_bench ALG LEN SECONDS T1 [T2 ...]
 *
 * Build: make -C tools coalesce_bench (links ilias_net2_amd/libnet2_sha2.so).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/uio.h>
#include <time.h>

#include "../include/net2/hash.h"

static int g_alg;
static size_t g_len;
static double g_secs;
static volatile int g_go;

struct worker {
	pthread_t tid;
	int idx;
	double *lat;		/* seconds per call */
	size_t nlat, cap;
	int rc;
};

static double now(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void *run(void *arg)
{
	struct worker *w = arg;
	uint8_t *msg = malloc(g_len ? g_len : 1), out[64], key[64];
	struct iovec v = { msg, g_len };
	size_t keylen = (size_t)net2_hash_getkeylen(g_alg);

	for (size_t i = 0; i < g_len; i++)
		msg[i] = (uint8_t)(i * 7 + w->idx);
	memset(key, 0x2a, sizeof(key));
	while (!g_go)
		;
	const double end = now() + g_secs;
	for (;;) {
		const double t0 = now();
		if (t0 >= end)
			break;
		msg[0] = (uint8_t)w->nlat;
		int rc = net2_hashctx_hashiov(g_alg, keylen ? key : NULL, keylen,
		    &v, 1, out, sizeof(out));
		const double t1 = now();
		if (rc != 0) {
			w->rc = rc;
			break;
		}
		if (w->nlat == w->cap) {
			w->cap = w->cap ? 2 * w->cap : 4096;
			w->lat = realloc(w->lat, w->cap * sizeof(double));
		}
		w->lat[w->nlat++] = t1 - t0;
	}
	free(msg);
	return NULL;
}

static int cmp(const void *a, const void *b)
{
	double x = *(const double *)a, y = *(const double *)b;
	return x < y ? -1 : x > y;
}

int main(int argc, char **argv)
{
	if (argc < 5) {
		fprintf(stderr, "usage: %s ALG LEN SECONDS T1 [T2 ...]\n", argv[0]);
		return 2;
	}
	g_alg = atoi(argv[1]);
	g_len = (size_t)atol(argv[2]);
	g_secs = atof(argv[3]);
	/* warm-up: device init, first staging allocation */
	{
		uint8_t m[64] = { 0 }, out[64], key[64] = { 0 };
		struct iovec v = { m, sizeof(m) };
		size_t kl = (size_t)net2_hash_getkeylen(g_alg);
		for (int i = 0; i < 200; i++) {
			int rc = net2_hashctx_hashiov(g_alg, kl ? key : NULL, kl, &v,
			    1, out, sizeof(out));
			if (rc != 0) {
				fprintf(stderr, "hashiov: %s\n", net2_sha2_strerror(rc));
				return 1;
			}
		}
	}
	for (int a = 4; a < argc; a++) {
		const int nt = atoi(argv[a]);
		struct worker *w = calloc((size_t)nt, sizeof(*w));
		g_go = 0;
		for (int t = 0; t < nt; t++) {
			w[t].idx = t;
			pthread_create(&w[t].tid, NULL, run, &w[t]);
		}
		const double t0 = now();
		g_go = 1;
		size_t total = 0;
		int rc = 0;
		for (int t = 0; t < nt; t++) {
			pthread_join(w[t].tid, NULL);
			total += w[t].nlat;
			if (w[t].rc)
				rc = w[t].rc;
		}
		const double el = now() - t0;
		double *all = malloc((total ? total : 1) * sizeof(double));
		size_t k = 0;
		for (int t = 0; t < nt; t++) {
			memcpy(all + k, w[t].lat, w[t].nlat * sizeof(double));
			k += w[t].nlat;
			free(w[t].lat);
		}
		qsort(all, total, sizeof(double), cmp);
		printf("{\"alg\": \"%s\", \"len\": %zu, \"threads\": %d, "
		    "\"calls\": %zu, \"msgs_per_s\": %.0f, \"median_us\": %.1f, "
		    "\"p99_us\": %.1f, \"min_us\": %.1f, \"rc\": %d}\n",
		    net2_hash_getname(g_alg), g_len, nt, total,
		    total / el, total ? all[total / 2] * 1e6 : 0.0,
		    total ? all[(size_t)(total * 0.99)] * 1e6 : 0.0,
		    total ? all[0] * 1e6 : 0.0, rc);
		fflush(stdout);
		free(all);
		free(w);
	}
	return 0;
}
