"""ilias_net2_amd -- MI355X-native batched SHA-2 for ilias_net2's integrity path.

Scope: the SHA-256/384/512 digests of src/sha2.c as
consumed by src/sign.c and src/signed_carver.c, computed by hand-written
gfx950 HIP kernels behind a C ABI (include/net2/*.h, libnet2_sha2.so).

* ``ilias_net2_amd.hash``  -- registry + ilias::hash factory mirror
* ``ilias_net2_amd.batch`` -- batched device / host digests
"""
from ._lib import (DIGEST_LEN, HMAC_SHA256, HMAC_SHA384, HMAC_SHA512, NIL,  # noqa: F401
                   SHA256, SHA384, SHA512, LIB_PATH, Net2Error, device_count,
                   lib)

__all__ = ["hash", "batch", "lib", "device_count", "Net2Error", "LIB_PATH",
           "SHA256", "SHA384", "SHA512", "HMAC_SHA256", "HMAC_SHA384",
           "HMAC_SHA512", "NIL", "DIGEST_LEN"]
