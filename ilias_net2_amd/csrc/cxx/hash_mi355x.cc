/*
 * hash_mi355x.cc -- MI355X backend of the reference's C++ hash interface
 * (include/ilias/net2/hash.h:31-79), the sibling of cxx_src/hash-openssl.cc:
 * the same six factories, names, lengths and key rules, with every
 * compression on the GPU.
 *
 *   factory.run(key, data)      -- one net2_hashctx_hashiov call over the
 *                                  buffer's segments (as hash-openssl.cc:
 *                                  235-237 visits them): one coalesced
 *                                  request, batched with concurrent callers;
 *   factory.instantiate(key)    -- a streaming context: the SHA2_CTX calls
 *     ->update(b) ... ->final()    of net2/sha2.h (SHA-256/384/512), or for
 *                                  HMAC an inner SHA2_CTX primed with
 *                                  K' ^ ipad and the outer hash at final().
 *
 * Key rules (hash-openssl.cc:199-200, 227-228, 383-386): an unkeyed factory
 * given a non-empty key throws std::invalid_argument("expected empty key
 * buffer for un-keyed hash"); a keyed one throws "key required" for an
 * empty key and "invalid key length" unless it has exactly keylen bytes.
 * A failed GPU call throws std::bad_alloc for ENOMEM, else
 * std::runtime_error naming the errno text.
 *
 * Built with -DILIAS_NET2_REFERENCE_TREE inside the reference tree (its own
 * hash.h / buffer.h); here against include/ilias_mi355x/hash_iface.h.
 */
#ifdef ILIAS_NET2_REFERENCE_TREE
#include <ilias/net2/buffer.h>
#include <ilias/net2/hash.h>
#else
#include "../../../include/ilias_mi355x/hash_iface.h"
#endif

#include "../../../include/net2/hash.h"
#include "../../../include/net2/sha2.h"

#include <errno.h>
#include <string.h>
#include <sys/uio.h>

#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#define NET2_CXX_EXPORT __attribute__((visibility("default")))

namespace ilias {
namespace {

void throw_for(int rc, const char *what)
{
	if (rc == 0)
		return;
	if (rc == ENOMEM)
		throw std::bad_alloc();
	throw std::runtime_error(std::string(what) + ": " +
	    net2_sha2_strerror(rc));
}

/* SHA-2 row of a registry row (HMAC-SHA* -> SHA*). */
int sha_row(int alg)
{
	return alg > NET2_HASH_SHA512 ? alg - 3 : alg;
}

/* Unkeyed: a SHA2_CTX whose compressions run on the GPU. */
class gpu_sha2_ctx : public hash_ctx {
public:
	gpu_sha2_ctx(int alg)
	    : hash_ctx(net2_hash_getname(alg), net2_hash_gethashlen(alg), 0),
	      alg_(alg)
	{
		throw_for(net2_sha2_ctx_init(alg_, &ctx_), "SHA2 init");
	}

	void update(const buffer &b) override
	{
		b.visit([this](const void *p, buffer::size_type l) {
			throw_for(net2_sha2_ctx_update(alg_, &ctx_, p, l),
			    "SHA2 update");
		});
	}

	buffer final() override
	{
		buffer rv;
		buffer::prepare prep(rv, hashlen);
		throw_for(net2_sha2_ctx_final(alg_,
		    static_cast<uint8_t *>(prep.data()), &ctx_), "SHA2 final");
		prep.commit();
		return rv;
	}

private:
	int alg_;
	SHA2_CTX ctx_;
};

/*
 * Keyed (RFC 2104): inner = H((K' ^ ipad) || m) streamed, outer =
 * H((K' ^ opad) || inner) at final(); K' = the key zero-padded to the block
 * (registry keys are never longer than a block).
 */
class gpu_hmac_ctx : public hash_ctx {
public:
	gpu_hmac_ctx(int alg, const void *key, size_t keylen)
	    : hash_ctx(net2_hash_getname(alg), net2_hash_gethashlen(alg),
		  net2_hash_getkeylen(alg)),
	      sha_(sha_row(alg)), blk_(sha_ == NET2_HASH_SHA256 ? 64 : 128)
	{
		memset(kpad_, 0, sizeof(kpad_));
		memcpy(kpad_, key, keylen);
		uint8_t ipad[128];
		for (size_t i = 0; i < blk_; i++)
			ipad[i] = kpad_[i] ^ 0x36;
		throw_for(net2_sha2_ctx_init(sha_, &inner_), "HMAC init");
		throw_for(net2_sha2_ctx_update(sha_, &inner_, ipad, blk_),
		    "HMAC init");
	}

	~gpu_hmac_ctx() noexcept override
	{
		memset(kpad_, 0, sizeof(kpad_));
		memset(&inner_, 0, sizeof(inner_));
	}

	void update(const buffer &b) override
	{
		b.visit([this](const void *p, buffer::size_type l) {
			throw_for(net2_sha2_ctx_update(sha_, &inner_, p, l),
			    "HMAC update");
		});
	}

	buffer final() override
	{
		uint8_t ih[64], opad[128];
		SHA2_CTX outer;
		throw_for(net2_sha2_ctx_final(sha_, ih, &inner_), "HMAC final");
		for (size_t i = 0; i < blk_; i++)
			opad[i] = kpad_[i] ^ 0x5c;
		buffer rv;
		buffer::prepare prep(rv, hashlen, true);
		throw_for(net2_sha2_ctx_init(sha_, &outer), "HMAC final");
		throw_for(net2_sha2_ctx_update(sha_, &outer, opad, blk_),
		    "HMAC final");
		throw_for(net2_sha2_ctx_update(sha_, &outer, ih, hashlen),
		    "HMAC final");
		throw_for(net2_sha2_ctx_final(sha_,
		    static_cast<uint8_t *>(prep.data()), &outer), "HMAC final");
		prep.commit();
		return rv;
	}

private:
	int sha_;
	size_t blk_;
	uint8_t kpad_[128];
	SHA2_CTX inner_;
};

class gpu_factory : public hash_ctx_factory {
public:
	explicit gpu_factory(int alg)
	    : hash_ctx_factory(net2_hash_getname(alg), net2_hash_gethashlen(alg),
		  net2_hash_getkeylen(alg)),
	      alg_(alg) {}

	hash_ctx_ptr instantiate(buffer key) const override
	{
		check_key(key);
		if (keylen == 0)
			return hash_ctx_ptr(new gpu_sha2_ctx(alg_));
		return hash_ctx_ptr(new gpu_hmac_ctx(alg_, key.pullup(),
		    key.size()));
	}

	/* The whole message as one request (hash-openssl.cc:224-282). */
	buffer run(buffer key, const buffer &data) const override
	{
		check_key(key);
		std::vector<struct iovec> iov;
		data.visit([&iov](const void *p, buffer::size_type l) {
			iov.push_back({ const_cast<void *>(p), (size_t)l });
		});
		const void *k = keylen ? key.pullup() : nullptr;
		buffer rv;
		buffer::prepare prep(rv, hashlen, keylen != 0);
		throw_for(net2_hashctx_hashiov(alg_, k, keylen ? key.size() : 0,
		    iov.data(), iov.size(), prep.data(), hashlen), name.c_str());
		prep.commit();
		return rv;
	}

private:
	void check_key(const buffer &key) const
	{
		if (keylen == 0) {
			if (!key.empty())
				throw std::invalid_argument(
				    "expected empty key buffer for un-keyed hash");
			return;
		}
		if (key.empty())
			throw std::invalid_argument("key required");
		if (key.size() != keylen)
			throw std::invalid_argument("invalid key length");
	}

	int alg_;
};

}	/* namespace */

namespace hash {

NET2_CXX_EXPORT const hash_ctx_factory &sha256()
{
	static const gpu_factory impl(NET2_HASH_SHA256);
	return impl;
}

NET2_CXX_EXPORT const hash_ctx_factory &sha384()
{
	static const gpu_factory impl(NET2_HASH_SHA384);
	return impl;
}

NET2_CXX_EXPORT const hash_ctx_factory &sha512()
{
	static const gpu_factory impl(NET2_HASH_SHA512);
	return impl;
}

NET2_CXX_EXPORT const hash_ctx_factory &hmac_sha256()
{
	static const gpu_factory impl(NET2_HASH_HMAC_SHA256);
	return impl;
}

NET2_CXX_EXPORT const hash_ctx_factory &hmac_sha384()
{
	static const gpu_factory impl(NET2_HASH_HMAC_SHA384);
	return impl;
}

NET2_CXX_EXPORT const hash_ctx_factory &hmac_sha512()
{
	static const gpu_factory impl(NET2_HASH_HMAC_SHA512);
	return impl;
}

}	/* namespace hash */
}	/* namespace ilias */
