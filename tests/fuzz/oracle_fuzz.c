/*
 * libFuzzer target for the CPU oracle (oracle/sha2_oracle.c), built with
 * AddressSanitizer and UBSan by tests/test_oracle.py.  Test infrastructure:
 * it checks the checker.  Per input:
 *   - SHA-256/384/512 one-shot == the streaming form fed in the input's own
 *     split points == OpenSSL's EVP digest;
 *   - HMAC-SHA256/384/512 under a key cut from the input == OpenSSL's HMAC;
 *   - the input as a received datagram: oracle_packet_decode_batch returns
 *     a code in 0..3 and touches nothing outside its arrays;
 *   - a datagram sealed by oracle_packet_encode_batch from the input's
 *     payload decodes NET2_PDECODE_OK with its header and the IV of
 *     oracle_ph_to_iv; with a bit of its hash field or payload flipped it
 *     decodes NET2_PDECODE_BAD, with a bit of its seq flipped still OK (the
 *     reference's HMAC does not cover the header).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <openssl/evp.h>
#include <openssl/hmac.h>

#include "../../oracle/sha2_oracle.h"

static const EVP_MD *
md_of(int alg)
{
	return alg == 1 ? EVP_sha256() : alg == 2 ? EVP_sha384() : EVP_sha512();
}

static void
check_digests(int alg, const uint8_t *m, size_t len, const uint8_t *cuts,
    size_t ncuts)
{
	uint8_t one[64], str[64], ref[64];
	unsigned int rl = 0;
	oracle_sha2_ctx c;
	size_t at = 0;
	int dl = oracle_sha2_digest(alg, m, len, one);

	if (alg == 1)
		oracle_sha256_init(&c);
	else if (alg == 2)
		oracle_sha384_init(&c);
	else
		oracle_sha512_init(&c);
	for (size_t k = 0; k <= ncuts; k++) {
		size_t step = k < ncuts ? cuts[k] : len - at;

		if (step > len - at)
			step = len - at;
		if (alg == 1)
			oracle_sha256_update(&c, m + at, step);
		else if (alg == 2)
			oracle_sha384_update(&c, m + at, step);
		else
			oracle_sha512_update(&c, m + at, step);
		at += step;
	}
	if (alg == 1)
		oracle_sha256_final(str, &c);
	else if (alg == 2)
		oracle_sha384_final(str, &c);
	else
		oracle_sha512_final(str, &c);
	if (!EVP_Digest(m, len, ref, &rl, md_of(alg), NULL) || (int)rl != dl ||
	    memcmp(one, ref, dl) != 0 || memcmp(str, ref, dl) != 0)
		abort();
}

static void
check_hmac(int alg, const uint8_t *key, size_t keylen, const uint8_t *m,
    size_t len)
{
	uint8_t out[64], ref[64];
	unsigned int rl = 0;
	int dl = oracle_hmac_digest(alg + 3, key, keylen, m, len, out);

	if (HMAC(md_of(alg), key, (int)keylen, m, len, ref, &rl) == NULL ||
	    (int)rl != dl || memcmp(out, ref, dl) != 0)
		abort();
}

static void
check_packet(const uint8_t *in, size_t len, int hash_alg, const uint8_t *key,
    size_t keylen, int enc_set)
{
	const size_t dlen = hash_alg == 4 ? 32 : hash_alg == 5 ? 48 : 64;
	uint64_t off = 0;
	uint32_t l32 = (uint32_t)len, seq = 0, flags = 0;
	uint8_t res = 0xee, iv[40], want[40];
	uint8_t *dg;

	/* the raw input as a received datagram */
	if (oracle_packet_decode_batch(hash_alg, key, keylen, NULL, 0, 0, 0, 0,
	    enc_set, sizeof(iv), in, &off, &l32, 1, &res, iv, &seq, &flags, 1) != 0 ||
	    res > 3)
		abort();

	/* a sealed datagram around the input's payload */
	if ((dg = malloc(8 + dlen + len)) == NULL)
		abort();
	memset(dg, 0xa5, 8 + dlen);
	if (len)
		memcpy(dg + 8, in, len);	/* payload after header + field */
	memmove(dg + 8 + dlen, dg + 8, len);
	seq = len >= 4 ? ((uint32_t)in[0] << 24 | (uint32_t)in[1] << 16 |
	    (uint32_t)in[2] << 8 | in[3]) : (uint32_t)len;
	flags = 0x2u | (enc_set ? 0x1u : 0u);	/* PH_SIGNED | PH_ENCRYPTED */
	l32 = (uint32_t)(8 + dlen + len);
	res = 0xee;
	if (oracle_packet_encode_batch(hash_alg, key, keylen, enc_set, &seq, &flags,
	    dg, &off, &l32, 1, &res, 1) != 0 || res != 0)
		abort();
	uint32_t s2 = 0, f2 = 0;
	res = 0xee;
	if (oracle_packet_decode_batch(hash_alg, key, keylen, NULL, 0, 0, 0, 0,
	    enc_set, sizeof(iv), dg, &off, &l32, 1, &res, iv, &s2, &f2, 1) != 0 ||
	    res != 0 || s2 != seq || f2 != flags)
		abort();
	if (enc_set) {
		if (oracle_ph_to_iv(seq, flags, sizeof(want), want) != 0 ||
		    memcmp(iv, want, sizeof(want)) != 0)
			abort();
	}
	/* the HMAC covers what follows the hash field, not the header
	 * (packet.n2t:232-257 hash the buffer left after both are removed):
	 * another seq still verifies, and is what decodes */
	dg[3] ^= 0x01;
	res = 0xee;
	if (oracle_packet_decode_batch(hash_alg, key, keylen, NULL, 0, 0, 0, 0,
	    enc_set, sizeof(iv), dg, &off, &l32, 1, &res, iv, &s2, &f2, 1) != 0 ||
	    res != 0 || s2 != (seq ^ 0x01u) || f2 != flags)
		abort();
	dg[3] ^= 0x01;
	/* one flipped bit in the hash field or the payload: NET2_PDECODE_BAD */
	size_t at = 8 + (len ? (size_t)in[0] * 131 : (size_t)seq) % (l32 - 8);
	dg[at] ^= 0x01;
	res = 0xee;
	if (oracle_packet_decode_batch(hash_alg, key, keylen, NULL, 0, 0, 0, 0,
	    enc_set, sizeof(iv), dg, &off, &l32, 1, &res, iv, &s2, &f2, 1) != 0 ||
	    res != 2)
		abort();
	free(dg);
}

int
LLVMFuzzerTestOneInput(const uint8_t *in, size_t len)
{
	if (len < 3)
		return 0;
	const int alg = 1 + in[0] % 3;
	const size_t keylen = in[1] % 200 < len - 2 ? in[1] % 200 : len - 2;
	const int enc_set = in[2] & 1;
	const uint8_t *key = in + 3 > in + len ? in : in + 3;
	const uint8_t *m = in + 3;
	size_t mlen = len - 3;

	check_digests(alg, m, mlen, in, len < 8 ? len : 8);
	check_hmac(alg, key, keylen < mlen ? keylen : mlen, m, mlen);
	check_packet(m, mlen, alg + 3, key, keylen < mlen ? keylen : mlen, enc_set);
	return 0;
}
