/*
 * libFuzzer target for the wire decoders of include/net2/wire.h (the bytes
 * a peer sends: types/signature.n2t:48-53, signed_carver_header.n2t:21-43),
 * built with AddressSanitizer and UBSan by tests/test_wire.py.  Test
 * infrastructure.  Every input that decodes must re-encode to exactly the
 * bytes consumed (the encoding is canonical: lengths, zero padding), and the
 * 4-byte carver header must round-trip.
 */
#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/net2/wire.h"

int
LLVMFuzzerTestOneInput(const uint8_t *in, size_t len)
{
	struct net2x_signature s;
	size_t used = 0;
	int rc = net2x_signature_decode(&s, in, len, &used);

	if (rc == 0) {
		size_t need = net2x_signature_encoded_len(&s), olen = need;
		uint8_t *out = malloc(need ? need : 1);

		if (out == NULL)
			abort();
		if (used > len || need != used ||
		    net2x_signature_encode(&s, out, &olen) != 0 || olen != used ||
		    memcmp(out, in, used) != 0)
			abort();
		free(out);
		net2x_signature_deinit(&s);
	} else if (rc != EINVAL) {
		abort();
	}
	if (len >= 4) {
		struct net2_signed_carver_header h;
		uint8_t back[4];

		net2_signed_carver_header_decode(&h, in);
		net2_signed_carver_header_encode(&h, back);
		if (memcmp(back, in, 4) != 0)
			abort();
	}
	return 0;
}
