/*
 * TEST INFRASTRUCTURE ONLY: a CPU baseline for bench.py's cpu_baseline leg,
 * never linked by the product.
 *
 * The reference's active C++ layer hashes through OpenSSL's low-level
 * SHA-2 calls -- SHA256_Init / SHA256_Update / SHA256_Final per message
 * (cxx_src/hash-openssl.cc:25-131, the hash_sha256 / hash_sha384 /
 * hash_sha512 contexts) -- not through src/sha2.c.  This times those same
 * library calls over a packet batch on the host, as context for the
 * src/sha2.c port the north star names: the system libcrypto
 * (OpenSSL 3.0.2 here) picks its own transform, SHA-NI / AVX2 where the
 * host has them.  Same batch layouts and slicing as oracle_sha2_batch.
 */
#define OPENSSL_SUPPRESS_DEPRECATED
#include <openssl/sha.h>
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>

struct ossl_slice {
	int alg;
	const uint8_t *base;
	const uint64_t *offsets;
	const uint32_t *lens;
	uint64_t stride;
	uint32_t fixed_len;
	size_t lo, hi;
	uint8_t *out;
};

static void *ossl_worker(void *arg)
{
	const struct ossl_slice *s = arg;
	static const size_t dlen_of[4] = { 0, 32, 48, 64 };
	const size_t dl = dlen_of[s->alg];
	for (size_t i = s->lo; i < s->hi; i++) {
		const uint8_t *p = s->offsets ? s->base + s->offsets[i] :
		    s->base + i * s->stride;
		const size_t len = s->offsets ? s->lens[i] : s->fixed_len;
		uint8_t *o = s->out + i * dl;
		if (s->alg == 1) {
			SHA256_CTX c;
			SHA256_Init(&c);
			SHA256_Update(&c, p, len);
			SHA256_Final(o, &c);
		} else {
			SHA512_CTX c;
			if (s->alg == 2)
				SHA384_Init(&c);
			else
				SHA512_Init(&c);
			SHA512_Update(&c, p, len);
			if (s->alg == 2)
				SHA384_Final(o, &c);
			else
				SHA512_Final(o, &c);
		}
	}
	return NULL;
}

/* alg 1/2/3 = SHA-256/384/512; 0 on success, -1 on a bad alg. */
int cpu_openssl_batch(int alg, const uint8_t *base, const uint64_t *offsets,
    const uint32_t *lens, uint64_t stride, uint32_t fixed_len, size_t n,
    uint8_t *out, int nthreads)
{
	struct ossl_slice sl[256];
	pthread_t tid[256];
	int t, started;

	if (alg < 1 || alg > 3)
		return -1;
	if (nthreads < 1)
		nthreads = 1;
	if (nthreads > 256)
		nthreads = 256;
	if ((size_t)nthreads > n)
		nthreads = n > 0 ? (int)n : 1;
	for (t = 0; t < nthreads; t++)
		sl[t] = (struct ossl_slice){ alg, base, offsets, lens, stride,
		    fixed_len, n * t / nthreads, n * (t + 1) / nthreads, out };
	if (nthreads == 1) {
		ossl_worker(&sl[0]);
		return 0;
	}
	for (started = 0; started < nthreads; started++)
		if (pthread_create(&tid[started], NULL, ossl_worker,
		    &sl[started]) != 0)
			break;
	for (t = started; t < nthreads; t++)
		ossl_worker(&sl[t]);
	for (t = 0; t < started; t++)
		pthread_join(tid[t], NULL);
	return 0;
}
