/*
 * test_hash.cc -- TEST INFRASTRUCTURE: the reference's C++ hash test
 * (test/hash.cc:50-80) restated against the MI355X backend
 * (ilias_net2_amd/csrc/cxx/hash_mi355x.cc), plus the key rules of
 * cxx_src/hash-openssl.cc and cross-checks against the CPU oracle
 * (oracle/sha2_oracle.c, linked as the checker only).
 *
 * Run by tests/test_cxx_hash.py (-m gpu); exits non-zero on the first
 * failure.
 */
#include "../../include/ilias_mi355x/hash_iface.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <stdexcept>
#include <string>

extern "C" {
int oracle_sha2_digest(int alg, const uint8_t *msg, size_t len, uint8_t *out);
int oracle_hmac_digest(int alg, const uint8_t *key, size_t keylen,
    const uint8_t *msg, size_t len, uint8_t *out);
}

#define TEST(x)                                                              \
	do {                                                                 \
		if (!(x)) {                                                  \
			fprintf(stderr, "%s:%d: test failed: %s\n", __FILE__,  \
			    __LINE__, #x);                                   \
			exit(1);                                             \
		}                                                            \
	} while (0)

static const char *father = "Luke, I am your father.";

/* test/hash.cc:23-48 (known answers, as data) */
static const char *father_hex[3] = {
	"5d8082c2eabfe36a513a644700155bc479ceee8533459e71678b689beabdd7d6",
	"ec2c17ed886aa29b3067690de319cfdcad69313e00390339d56dfec13dde384b"
	"f06342cdf9f58ffb5a9fcdfcc9db3c93",
	"9759a18565f81720c112d84041ec1aa23196378d27cfe0f47ad35d0afad58421"
	"3846f46f50994168ed0993be1193dc592b1a04f0404b9df587175974c97a1ffe",
};

static ilias::buffer from_hex(const char *h)
{
	std::string b;
	for (size_t i = 0; h[i] && h[i + 1]; i += 2)
		b.push_back((char)std::stoi(std::string(h + i, 2), nullptr, 16));
	return ilias::buffer(b.data(), b.size());
}

static ilias::buffer bytes(const std::string &s)
{
	return ilias::buffer(s.data(), s.size());
}

/* test/hash.cc:50-67: run() and instantiate -> update -> final agree with
 * the expected digest */
static void test_hash(const ilias::hash_ctx_factory &f,
    const ilias::buffer &in, const ilias::buffer &expect)
{
	printf("Test algorithm: %s\n", f.name.c_str());
	printf("- automatic hash_ctx_factory run...\n");
	TEST(f.run(ilias::buffer(), in) == expect);
	printf("- manual hash_ctx_factory run...\n");
	const ilias::hash_ctx_ptr hp = f.instantiate(ilias::buffer());
	hp->update(in);
	TEST(hp->final() == expect);
}

template <class F>
static bool throws_invalid(F f, const char *msg)
{
	try {
		f();
	} catch (const std::invalid_argument &e) {
		return strcmp(e.what(), msg) == 0;
	}
	return false;
}

int main()
{
	const ilias::buffer in(father, strlen(father));
	const ilias::hash_ctx_factory *unkeyed[3] = { &ilias::hash::sha256(),
	    &ilias::hash::sha384(), &ilias::hash::sha512() };
	const ilias::hash_ctx_factory *keyed[3] = { &ilias::hash::hmac_sha256(),
	    &ilias::hash::hmac_sha384(), &ilias::hash::hmac_sha512() };

	for (int a = 0; a < 3; a++)
		test_hash(*unkeyed[a], in, from_hex(father_hex[a]));

	/* names and lengths (hash-openssl.cc:139,154,169, 417-429) */
	TEST(unkeyed[0]->name == "SHA256" && unkeyed[0]->hashlen == 32 &&
	    unkeyed[0]->keylen == 0);
	TEST(keyed[2]->name == "HMAC-SHA512" && keyed[2]->hashlen == 64 &&
	    keyed[2]->keylen == 64);

	/* key rules (hash-openssl.cc:199-200, 227-228, 383-386) */
	TEST(throws_invalid([&]() { unkeyed[1]->run(bytes("k"), in); },
	    "expected empty key buffer for un-keyed hash"));
	TEST(throws_invalid([&]() { unkeyed[2]->instantiate(bytes("k")); },
	    "expected empty key buffer for un-keyed hash"));
	TEST(throws_invalid([&]() { keyed[0]->instantiate(ilias::buffer()); },
	    "key required"));
	TEST(throws_invalid([&]() { keyed[1]->run(bytes("short"), in); },
	    "invalid key length"));

	/* RFC 4231 case 2 ("Jefe"), the key zero-extended to the registry's
	 * key length (RFC 2104 pads K with zeros to the block) */
	static const char *jefe[3] = {
		"5bdcc146bf60754e6a042426089575c75a003f089d2739839dec58b964ec3843",
		"af45d2e376484031617f78d2b58a6b1b9c7ef464f5a01b47e42ec3736322445e"
		"8e2240ca5e69e2c78b3239ecfab21649",
		"164b7a7bfcf819e2e395fbe73b56e0a387bd64222e831fd610270cd7ea250554"
		"9758bf75c05a994a6d034f65f8f0e6fdcaeab1a34d4a6b4b636e070a38bce737",
	};
	const ilias::buffer what = bytes("what do ya want for nothing?");
	for (int a = 0; a < 3; a++) {
		std::string k("Jefe");
		k.resize(keyed[a]->keylen, '\0');
		TEST(keyed[a]->run(bytes(k), what) == from_hex(jefe[a]));
		auto c = keyed[a]->instantiate(bytes(k));
		c->update(bytes("what do ya "));
		c->update(bytes("want for nothing?"));
		TEST(c->final() == from_hex(jefe[a]));
	}

	/* random messages in several segments: run(), streamed updates and
	 * the oracle agree, for every row */
	std::mt19937 rng(7);
	for (int iter = 0; iter < 40; iter++) {
		const size_t n = rng() % 5000;
		std::string m(n, '\0');
		for (auto &c : m)
			c = (char)rng();
		ilias::buffer msg;
		for (size_t at = 0; at < n;) {
			size_t take = std::min<size_t>(n - at, 1 + rng() % 700);
			msg += ilias::buffer(m.data() + at, take);
			at += take;
		}
		TEST(msg.size() == n);
		const uint8_t *mp = (const uint8_t *)m.data();
		for (int a = 0; a < 3; a++) {
			uint8_t want[64];
			const int dl = oracle_sha2_digest(a + 1, mp, n, want);
			const ilias::buffer w(want, dl);
			TEST(unkeyed[a]->run(ilias::buffer(), msg) == w);
			auto c = unkeyed[a]->instantiate(ilias::buffer());
			c->update(msg);
			TEST(c->final() == w);

			std::string k(keyed[a]->keylen, '\0');
			for (auto &ch : k)
				ch = (char)rng();
			const int hl = oracle_hmac_digest(a + 4,
			    (const uint8_t *)k.data(), k.size(), mp, n, want);
			const ilias::buffer wh(want, hl);
			TEST(keyed[a]->run(bytes(k), msg) == wh);
			auto h = keyed[a]->instantiate(bytes(k));
			h->update(msg);
			TEST(h->final() == wh);
		}
	}
	printf("test_hash: ok\n");
	return 0;
}
