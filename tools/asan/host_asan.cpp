/*
 * host_asan -- the host side of libnet2_sha2 under AddressSanitizer (test
 * infrastructure, built by tools/asan/Makefile: every object of the library
 * recompiled with ASan on the host code only, the device code unchanged,
 * linked into this executable together with the CPU oracle as the checker).
 *
 * Drives the host pipelines a caller reaches through the C ABI and checks
 * every output against the oracle:
 *   net2_sha2_batch           fixed and variable layouts, pageable and
 *                             page-locked, 0 .. 2 chunks, ragged lengths;
 *   net2_packet_*_burst_host  TX then RX (tampered bytes, runts, unsigned
 *                             datagrams) at the wave-form, lane-form and
 *                             binned sizes, pageable and page-locked;
 *   net2_hashctx_hashiov      single calls from 8 threads at once (the
 *                             coalescer);
 * then the argument checks (EINVAL before any device work).
 * Prints "host_asan ok" and exits 0 when everything matched; ASan aborts
 * the process on a heap, stack or global overflow or a use after free.  A
 * watchdog reports each single-call thread's last call and exits 3 if the
 * single calls take more than 20 s.
 *
 *   NET2_SHA2_VIRTUAL_DEVICES=3 ./host_asan   also runs the sharded paths
 */
#include <hip/hip_runtime_api.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <unistd.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/net2/hash.h"
#include "../../include/net2/packet.h"
#include "../../include/net2/sha2_batch.h"
#include "../../oracle/sha2_oracle.h"

static int failures;

#define CHECK(c, ...) do { if (!(c)) { failures++; \
	fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
	fprintf(stderr, __VA_ARGS__); fputc('\n', stderr); } } while (0)

static uint64_t rng_state = 0x9e3779b97f4a7c15ull;
static uint64_t rnd()
{
	uint64_t x = rng_state;
	x ^= x >> 12; x ^= x << 25; x ^= x >> 27;
	rng_state = x;
	return x * 0x2545f4914f6cdd1dull;
}

/* Host memory of one kind: pageable (std::vector) or page-locked. */
template <class T> struct Buf {
	T *p = nullptr;
	size_t n = 0;
	bool pinned = false;
	std::vector<T> v;
	Buf(size_t n_, bool pin) : n(n_), pinned(pin) {
		if (pin) {
			if (hipHostMalloc((void **)&p, (n ? n : 1) * sizeof(T), 0) != hipSuccess) {
				fprintf(stderr, "hipHostMalloc failed\n");
				exit(2);
			}
		} else {
			v.resize(n ? n : 1);
			p = v.data();
		}
	}
	~Buf() { if (pinned) (void)hipHostFree(p); }
	Buf(const Buf &) = delete;
	Buf &operator=(const Buf &) = delete;
	T &operator[](size_t i) { return p[i]; }
};

static int dlen_of(int alg) { return alg == 1 ? 32 : alg == 2 ? 48 : 64; }

static void batch_case(int alg, bool var, uint64_t n, uint32_t maxlen, bool pin)
{
	const int dl = dlen_of(alg);
	std::vector<uint64_t> offs(n ? n : 1);
	std::vector<uint32_t> lens(n ? n : 1);
	uint64_t total = 0;
	const uint32_t fixed = maxlen;
	const uint64_t stride = (uint64_t)fixed + 7;	/* not 16-byte aligned */
	for (uint64_t i = 0; i < n; i++) {
		if (var) {
			lens[i] = (uint32_t)(rnd() % (maxlen + 1));
			offs[i] = total;
			total += lens[i] + (rnd() % 5);
		}
	}
	if (!var)
		total = n ? (n - 1) * stride + fixed : 0;
	Buf<uint8_t> data(total, pin), dig((size_t)n * dl, pin);
	for (uint64_t i = 0; i < total; i++)
		data[i] = (uint8_t)rnd();
	std::vector<uint8_t> want((size_t)n * dl + 1);
	int rc = var
	    ? net2_sha2_batch(alg, data.p, offs.data(), lens.data(), 0, 0, n, dig.p, 0)
	    : net2_sha2_batch(alg, data.p, nullptr, nullptr, stride, fixed, n, dig.p, 0);
	CHECK(rc == 0, "net2_sha2_batch alg %d var %d n %llu pin %d: rc %d", alg, var,
	    (unsigned long long)n, pin, rc);
	if (n == 0)
		return;
	if (var)
		oracle_sha2_batch(alg, data.p, offs.data(), lens.data(), 0, 0, n,
		    want.data(), 8);
	else
		oracle_sha2_batch(alg, data.p, nullptr, nullptr, stride, fixed, n,
		    want.data(), 8);
	CHECK(memcmp(dig.p, want.data(), (size_t)n * dl) == 0,
	    "digests differ: alg %d var %d n %llu pin %d", alg, var,
	    (unsigned long long)n, pin);
}

static void burst_case(int hash_alg, bool enc, uint32_t ivlen, uint64_t n, bool pin)
{
	fprintf(stderr, "burst alg %d n %llu pin %d\n", hash_alg,
	    (unsigned long long)n, pin);
	const uint32_t hl = (uint32_t)dlen_of(hash_alg - 3);
	std::vector<uint32_t> seq(n ? n : 1), fl(n ? n : 1), slot(n ? n : 1);
	std::vector<uint64_t> offs(n ? n : 1);
	static const uint32_t plens[] = {0, 1, 55, 56, 111, 112, 119, 120, 127, 128,
	    500, 1428};
	uint64_t total = 0;
	for (uint64_t i = 0; i < n; i++) {
		seq[i] = (uint32_t)rnd();
		fl[i] = NET2_PH_SIGNED | (enc ? NET2_PH_ENCRYPTED : 0);
		if (rnd() % 16 == 0)
			fl[i] ^= NET2_PH_SIGNED;
		slot[i] = 8 + hl + plens[rnd() % 12];
		if (rnd() % 25 == 0)
			slot[i] = (uint32_t)(rnd() % (8 + hl + 1));	/* no room */
		offs[i] = total;
		total += slot[i] + rnd() % 5;
	}
	std::vector<uint8_t> key(hl);
	for (auto &b : key)
		b = (uint8_t)rnd();
	Buf<uint8_t> buf(total, pin);
	for (uint64_t i = 0; i < total; i++)
		buf[i] = (uint8_t)rnd();
	std::vector<uint8_t> sealed(buf.p, buf.p + total), o_res(n ? n : 1);

	/* TX */
	Buf<uint8_t> res(n, pin);
	int rc = net2_packet_encode_burst_host(hash_alg, key.data(), hl, enc,
	    seq.data(), fl.data(), buf.p, offs.data(), slot.data(), n, res.p, 0);
	CHECK(rc == 0, "encode_burst_host n %llu: rc %d", (unsigned long long)n, rc);
	oracle_packet_encode_batch(hash_alg, key.data(), hl, enc, seq.data(),
	    fl.data(), sealed.data(), offs.data(), slot.data(), n, o_res.data(), 8);
	CHECK(n == 0 || (memcmp(res.p, o_res.data(), n) == 0 &&
	    memcmp(buf.p, sealed.data(), total) == 0),
	    "TX differs: n %llu pin %d", (unsigned long long)n, pin);

	/* RX: tamper, cut runts */
	std::vector<uint32_t> lens(slot);
	for (uint64_t i = 0; i < n; i++) {
		uint64_t t = rnd() % 100;
		if (t < 10 && lens[i] > 8)
			buf[offs[i] + 8 + rnd() % (lens[i] - 8)] ^= 0x10;
		else if (t < 13)
			lens[i] = 5;
	}
	const uint32_t ivb = ivlen ? ivlen : 1;
	Buf<uint8_t> r2(n, pin), iv((size_t)n * ivb, pin);
	Buf<uint32_t> s2(n, pin), f2(n, pin);
	memset(r2.p, 9, n ? n : 1);
	memset(iv.p, 0, (size_t)(n ? n : 1) * ivb);
	struct net2_burst_rx_keys k = {};
	k.hash_alg = hash_alg;
	k.hash_key = key.data();
	k.hash_keylen = hl;
	k.enc_alg = enc ? 1 : 0;
	fprintf(stderr, "  tx ok, rx\n");
	rc = net2_packet_decode_burst_host(&k, ivlen, buf.p, offs.data(),
	    lens.data(), n, r2.p, ivlen ? iv.p : nullptr, s2.p, f2.p, 0);
	CHECK(rc == 0, "decode_burst_host n %llu: rc %d", (unsigned long long)n, rc);
	std::vector<uint8_t> w_res(n ? n : 1), w_iv((size_t)(n ? n : 1) * ivb);
	std::vector<uint32_t> w_s(n ? n : 1), w_f(n ? n : 1);
	oracle_packet_decode_batch(hash_alg, key.data(), hl, nullptr, 0, 0, 0, 0,
	    enc, ivlen, buf.p, offs.data(), lens.data(), n, w_res.data(),
	    ivlen ? w_iv.data() : nullptr, w_s.data(), w_f.data(), 8);
	uint64_t bad = 0;
	for (uint64_t i = 0; i < n; i++) {
		bool same = r2[i] == w_res[i] && (r2[i] != 0 ||
		    (s2[i] == w_s[i] && f2[i] == w_f[i]));
		if (same && r2[i] == 0 && ivlen && (w_f[i] & NET2_PH_ENCRYPTED))
			same = memcmp(iv.p + i * ivb, w_iv.data() + i * ivb, ivlen) == 0;
		bad += !same;
	}
	CHECK(bad == 0, "RX differs at %llu of %llu datagrams (pin %d)",
	    (unsigned long long)bad, (unsigned long long)n, pin);
}

/* what each single-call thread is doing (a watchdog reports it if the
 * calls do not finish) */
static std::atomic<int> sc_state[8][3];	/* call index, alg, length */
static std::atomic<bool> sc_done{false};

static void single_calls()
{
	std::vector<std::thread> th;
	std::vector<int> bad(8, 0);
	std::thread dog([] {
		for (int i = 0; i < 400 && !sc_done.load(); i++)
			std::this_thread::sleep_for(std::chrono::milliseconds(50));
		if (sc_done.load())
			return;
		uint64_t calls = 0, launches = 0;
		net2_coalesce_stats(0, &calls, &launches);
		fprintf(stderr, "watchdog: single calls not done after 20 s; "
		    "coalescer calls %llu launches %llu\n",
		    (unsigned long long)calls, (unsigned long long)launches);
		for (int t = 0; t < 8; t++)
			fprintf(stderr, "  thread %d: call %d alg %d len %d\n", t,
			    sc_state[t][0].load(), sc_state[t][1].load(),
			    sc_state[t][2].load());
		_exit(3);
	});
	for (int t = 0; t < 8; t++)
		th.emplace_back([t, &bad] {
			uint64_t s = 0x1234567ull * (t + 1);
			for (int c = 0; c < 150; c++) {
				s = s * 6364136223846793005ull + 1442695040888963407ull;
				const int alg = 1 + (int)((s >> 33) % 6);	/* 1..3, HMAC 4..6 */
				const size_t len = (size_t)((s >> 20) % 3000);
				/* an HMAC row takes a key of its registry length */
				std::vector<uint8_t> m(len + 1),
				    key(alg > 3 ? (size_t)net2_hash_getkeylen(alg) : 1);
				for (size_t i = 0; i < len; i++)
					m[i] = (uint8_t)(s >> (i % 56));
				for (size_t i = 0; i < key.size(); i++)
					key[i] = (uint8_t)(i * 7 + t);
				const size_t cut = len / 3;
				struct iovec iov[2] = {{m.data(), cut}, {m.data() + cut, len - cut}};
				uint8_t out[64], want[64];
				const bool hm = alg > 3;
				sc_state[t][0] = c;
				sc_state[t][1] = alg;
				sc_state[t][2] = (int)len;
				int rc = net2_hashctx_hashiov(alg, hm ? key.data() : nullptr,
				    hm ? key.size() : 0, iov, 2, out, sizeof(out));
				int dl = hm ? oracle_hmac_digest(alg, key.data(), key.size(),
				    m.data(), len, want) : oracle_sha2_digest(alg, m.data(), len, want);
				if (rc != 0 || memcmp(out, want, dl) != 0)
					bad[t]++;
			}
		});
	for (auto &x : th)
		x.join();
	sc_done = true;
	dog.join();
	int sum = 0;
	for (int b : bad)
		sum += b;
	CHECK(sum == 0, "%d single calls differ", sum);
}

static void argument_checks()
{
	uint8_t d[64];
	uint64_t off = 0;
	uint32_t len = 4;
	CHECK(net2_sha2_batch(9, d, nullptr, nullptr, 64, 64, 1, d, 0) == EINVAL,
	    "unknown alg accepted");
	CHECK(net2_sha2_batch(1, nullptr, nullptr, nullptr, 64, 64, 1, d, 0) == EINVAL,
	    "NULL base accepted");
	CHECK(net2_sha2_batch(1, d, &off, nullptr, 0, 0, 1, d, 0) == EINVAL,
	    "offsets without lens accepted");
	CHECK(net2_sha2_batch(1, d, nullptr, nullptr, 8, 64, 2, d, 0) == EINVAL,
	    "stride below the packet length accepted");
	uint8_t r;
	CHECK(net2_packet_decode_burst_host(nullptr, 0, d, &off, &len, 1, &r,
	    nullptr, nullptr, nullptr, 0) == EINVAL, "NULL keys accepted");
	struct net2_burst_rx_keys k = {};
	k.hash_alg = 6;
	k.hash_key = d;
	k.hash_keylen = 3;		/* not the registry's key length */
	CHECK(net2_packet_decode_burst_host(&k, 0, d, &off, &len, 1, &r, nullptr,
	    nullptr, nullptr, 0) == EINVAL, "short HMAC key accepted");
}

int main()
{
	int ndev = 0;
	if (net2_sha2_device_count(&ndev) != 0 || ndev < 1) {
		fprintf(stderr, "host_asan: no gfx950 device\n");
		return 77;
	}
	for (int pin = 0; pin < 2; pin++) {
		batch_case(1, false, 0, 1024, pin);
		batch_case(1, false, 1, 1024, pin);
		batch_case(3, false, 1000, 1024, pin);
		batch_case(1, false, 70000, 1024, pin);		/* two 64 MiB chunks */
		batch_case(1, true, 5000, 1600, pin);
		batch_case(2, true, 150000, 1100, pin);		/* binned, two chunks */
	}
	fprintf(stderr, "batches done (%d failures)\n", failures);
	for (int pin = 0; pin < 2; pin++) {
		burst_case(6, true, 16, 1, pin);
		burst_case(6, true, 16, 64, pin);		/* wave form */
		burst_case(4, true, 32, 5000, pin);
		burst_case(5, false, 0, 20000, pin);		/* lane form, unbinned */
		burst_case(6, true, 16, 70000, pin);		/* binned */
	}
	fprintf(stderr, "bursts done (%d failures)\n", failures);
	single_calls();
	argument_checks();
	if (failures) {
		fprintf(stderr, "host_asan: %d failures\n", failures);
		return 1;
	}
	printf("host_asan ok\n");
	return 0;
}
