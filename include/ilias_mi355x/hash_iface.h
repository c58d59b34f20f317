/*
 * ilias_mi355x/hash_iface.h -- the C++ hash interface of the reference's
 * active build, restated so the MI355X backend (csrc/cxx/hash_mi355x.cc)
 * builds and is tested in this repository.
 *
 * Interface being restated: include/ilias/net2/hash.h:31-79 (class
 * ilias::hash_ctx with hashlen / keylen / name, update(const buffer&),
 * final(); class ilias::hash_ctx_factory with instantiate(buffer) and
 * run(buffer key, const buffer& data); the six factories of namespace
 * ilias::hash) and the part of ilias::buffer those signatures and the
 * backends use (include/ilias/net2/buffer.h: the (data, len) constructor
 * :784, size() :796, operator== :919, visit(f) :958-970, pullup() :1058,
 * buffer::prepare :1143-1216).
 *
 * Inside the reference tree the backend is compiled with
 * -DILIAS_NET2_REFERENCE_TREE and includes the reference's own
 * <ilias/net2/hash.h> and <ilias/net2/buffer.h> instead of this file
 * (INTEGRATION.md).  Here `buffer` is a plain list of byte segments.
 */
#ifndef ILIAS_MI355X_HASH_IFACE_H
#define ILIAS_MI355X_HASH_IFACE_H

#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace ilias {

/* Byte segments, shared on copy like the reference's segment refs. */
class buffer {
public:
	typedef uintptr_t size_type;
	class prepare;

	buffer() = default;
	buffer(const void *data, size_type len)
	{
		if (len > 0)
			segs_.push_back(std::make_shared<std::vector<uint8_t>>(
			    static_cast<const uint8_t *>(data),
			    static_cast<const uint8_t *>(data) + len));
	}

	size_type size() const noexcept
	{
		size_type n = 0;
		for (const auto &s : segs_)
			n += s->size();
		return n;
	}
	bool empty() const noexcept { return size() == 0; }
	size_type segments() const noexcept { return segs_.size(); }

	/* Append o's segments (no copy of their bytes). */
	buffer &operator+=(const buffer &o)
	{
		segs_.insert(segs_.end(), o.segs_.begin(), o.segs_.end());
		return *this;
	}

	/* f(const void *, size_type) for every segment, in order. */
	template <class F>
	void visit(F f) const
	{
		for (const auto &s : segs_)
			f(static_cast<const void *>(s->data()), s->size());
	}

	/* Contiguous view of the whole buffer (merges the segments). */
	const void *pullup()
	{
		if (segs_.size() > 1) {
			auto all = std::make_shared<std::vector<uint8_t>>();
			for (const auto &s : segs_)
				all->insert(all->end(), s->begin(), s->end());
			segs_.assign(1, all);
		}
		return segs_.empty() ? nullptr : segs_[0]->data();
	}

	bool operator==(const buffer &o) const noexcept
	{
		std::vector<uint8_t> a, b;
		visit([&a](const void *p, size_type l) {
			a.insert(a.end(), (const uint8_t *)p, (const uint8_t *)p + l);
		});
		o.visit([&b](const void *p, size_type l) {
			b.insert(b.end(), (const uint8_t *)p, (const uint8_t *)p + l);
		});
		return a == b;
	}
	bool operator!=(const buffer &o) const noexcept { return !(*this == o); }

private:
	std::vector<std::shared_ptr<std::vector<uint8_t>>> segs_;
};

/* Reserve len bytes at the back of b; they join b on commit(). */
class buffer::prepare {
public:
	prepare(buffer &b, size_type len, bool sensitive = false)
	    : b_(&b), seg_(std::make_shared<std::vector<uint8_t>>(len))
	{
		(void)sensitive;
	}
	void *data(size_type off = 0) const noexcept
	{
		return off < seg_->size() ? seg_->data() + off : nullptr;
	}
	size_type size() const noexcept { return seg_->size(); }
	void commit() noexcept
	{
		if (b_ != nullptr && !seg_->empty())
			b_->segs_.push_back(seg_);
		b_ = nullptr;
	}

private:
	buffer *b_;
	std::shared_ptr<std::vector<uint8_t>> seg_;
};

/* One hash computation in progress. */
class hash_ctx {
public:
	typedef std::uint32_t size_type;

	const size_type hashlen;
	const size_type keylen;
	const std::string name;

	hash_ctx(std::string n, size_type hl, size_type kl)
	    : hashlen(hl), keylen(kl), name(std::move(n)) {}
	virtual ~hash_ctx() noexcept {}

	virtual void update(const buffer &) = 0;
	virtual buffer final() = 0;
};

typedef std::unique_ptr<hash_ctx> hash_ctx_ptr;

/* An algorithm of the registry: makes contexts, or hashes in one go. */
class hash_ctx_factory {
public:
	typedef hash_ctx::size_type size_type;

	const size_type hashlen;
	const size_type keylen;
	const std::string name;

	hash_ctx_factory(std::string n, size_type hl, size_type kl)
	    : hashlen(hl), keylen(kl), name(std::move(n)) {}
	virtual ~hash_ctx_factory() noexcept {}

	virtual hash_ctx_ptr instantiate(buffer key) const = 0;

	/* instantiate(key), update(data), final() (cxx_src/hash.cc:42-48) */
	virtual buffer run(buffer key, const buffer &data) const
	{
		hash_ctx_ptr c = instantiate(std::move(key));
		c->update(data);
		return c->final();
	}
};

namespace hash {

const hash_ctx_factory &sha256();
const hash_ctx_factory &sha384();
const hash_ctx_factory &sha512();
const hash_ctx_factory &hmac_sha256();
const hash_ctx_factory &hmac_sha384();
const hash_ctx_factory &hmac_sha512();

}	/* namespace hash */
}	/* namespace ilias */

#endif /* ILIAS_MI355X_HASH_IFACE_H */
