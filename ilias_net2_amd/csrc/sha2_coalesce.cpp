/*
 * sha2_coalesce.cpp -- request coalescer for the single-message paths
 * (see sha2_coalesce.h).
 *
 * Per device: a few batch slots, each with pinned host staging, device
 * staging, a stream and an event.  One slot at a time is "open": callers
 * reserve a range of its staging under the device mutex, copy and pad their
 * message outside it, and wait.  The first caller of a batch leads it:
 *   - it launches at once if no other batch of this device is in flight
 *     (an idle GPU: lowest latency for a lone caller),
 *   - otherwise when the batch is full or the batching window (default
 *     20 us, NET2_COALESCE_WINDOW_US) has passed since it opened -- the
 *     callers that arrive while earlier batches run share one launch
 *     (20 us measured best over 10 / 20 / 40 / 80 us at 8 and 64 threads,
 *     profiles/round2/coalesce_window_ab.txt);
 * then it waits for the batch's event (spinning briefly, then blocking) and
 * hands every caller its result.  Several batches may be in flight at once
 * (NET2_COALESCE_SLOTS, default 8: ahead of 4 at 64 and 128 threads, even
 * at 8, profiles/round2/coalesce_slots_ab.txt), each on its own stream.
 *
 * Layout of a batch in staging: every job's blocks (the message already
 * padded as SHA*Pad would, src/sha2.c:495-543 / :784-832, behind the
 * K' ^ ipad block for HMAC), then its aux block (K' ^ opad, or the state to
 * continue from), each job 64-byte aligned; at launch the leader appends
 * the job descriptors.  Results: 64 bytes of raw state per job.
 */
#include "sha2_coalesce.h"
#include "sha2_launch.h"

#include <hip/hip_runtime.h>

#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <vector>

namespace net2co {
namespace {

typedef std::chrono::steady_clock clk;

constexpr int kMaxSlots = 16;
constexpr size_t kInitialStage = 1u << 20;	/* grows on demand */
/* staging grown past this is released lazily: when a later batch on the
 * same slot uses under a quarter of it.  A run of large requests (the
 * 64 MiB pieces of a long SHA*Update or streamed hashiov, repeated 32 MiB
 * calls) keeps reusing the slot's staging -- free slots are taken
 * last-in-first-out, so a serial caller gets the same slot back -- instead
 * of page-locking and freeing ~80 MiB per request (hipHostFree / hipFree
 * also synchronise the device, stalling other slots' batches); the first
 * small batch afterwards gives it back, so a few big calls do not keep
 * gigabytes page-locked for the life of the process */
constexpr size_t kRetainStage = 16u << 20;
constexpr size_t kMaxJobs = 1u << 16;		/* per batch */
/*
 * Up to this many jobs a batch runs one wave per job (job_wave_kernel, the
 * latency form); larger batches one lane per job.  Measured with
 * tools/coalesce_bench.c, 1 KiB messages (profiles/round2/coalesce_jm*):
 * the wave form cuts a lone call from 82 to 50 us (SHA-512) and 64 to
 * 55 us (SHA-256) and wins at 8 threads; at 64 threads, where batches
 * hold tens of jobs, the lane form keeps up equally (SHA-512) or better
 * (SHA-256: 433 k vs 349 k calls/s).
 */
constexpr size_t kWaveJobsMax = 16;
/* ... and any job this long takes the wave form whatever the batch size: in
 * the lane form one lane runs every compression of its job in turn, a
 * 4 GiB message for minutes (64 KiB of SHA-256, 128 KiB of SHA-512) */
constexpr uint32_t kWaveBlocks = 1024;

int env_int(const char *name, int dflt, int lo, int hi)
{
	const char *v = getenv(name);
	if (v == nullptr || *v == '\0')
		return dflt;
	return std::min(hi, std::max(lo, atoi(v)));
}

size_t align64(size_t x)
{
	return (x + 63) & ~(size_t)63;
}

struct Job {
	Net2Job desc;		/* offsets relative to the slot's staging */
	int kind, alg;
	uint8_t *out;
	std::atomic<int> done{0};
	int rc = 0;
	int hip = 0;		/* HIP error behind rc == EIO */
};

struct Slot {
	hipStream_t stream = nullptr;
	hipEvent_t ev = nullptr;
	uint8_t *h_stage = nullptr, *d_stage = nullptr;
	size_t cap = 0;
	uint8_t *h_out = nullptr;	/* coherent, written by the kernel */
	size_t cap_jobs = 0;
	/* the batch being filled or run */
	std::vector<Job *> jobs;
	size_t used = 0;
	std::atomic<int> writers{0};	/* reservations still being filled */
	bool full = false;
	/* completion: every wave of the batch's launches adds 1 here (host
	 * memory, written by the GPU) once its results are stored */
	uint32_t *h_done = nullptr;
	uint32_t done_base = 0;
	clk::time_point opened;

	void free_stage()
	{
		if (h_stage) (void)hipHostFree(h_stage);
		if (d_stage && d_stage != h_stage) (void)hipFree(d_stage);
		h_stage = d_stage = nullptr;
		cap = 0;
	}
	void free_out()
	{
		if (h_out) (void)hipHostFree(h_out);
		h_out = nullptr;
		cap_jobs = 0;
	}
};

/*
 * zerocopy (default): the kernel reads the staging through the host mapping
 * of a coherent pinned buffer, so a batch costs one kernel launch and no
 * copy; NET2_COALESCE_ZEROCOPY=0 copies the staging to device memory first.
 * With the wave-per-job form the copy and its dependency cost more than
 * the kernel's reads over PCIe: a lone 1 KiB call 48.5 against 51.1 us
 * (SHA-512), 64 threads 385 k against 373 k calls/s (SHA-256: 453 k against
 * 427 k), profiles/round2/coalesce_zc_ab.txt.  (Results always come back
 * through coherent host memory written by the kernel.)
 */
hipError_t host_alloc(uint8_t **p, size_t bytes, bool zerocopy)
{
	return hipHostMalloc((void **)p, bytes, zerocopy ?
	    (hipHostMallocMapped | hipHostMallocCoherent) : hipHostMallocDefault);
}

/* Linux futex on a job's completion word: the leader wakes exactly the
 * callers of its batch (a shared condition variable woke every waiting
 * thread on every completion, and they queued on one mutex). */
void futex_wait(std::atomic<int> *w, int val)
{
	syscall(SYS_futex, reinterpret_cast<int *>(w), FUTEX_WAIT_PRIVATE, val,
	    nullptr, nullptr, 0);
}

void futex_wake(std::atomic<int> *w)
{
	syscall(SYS_futex, reinterpret_cast<int *>(w), FUTEX_WAKE_PRIVATE,
	    INT32_MAX, nullptr, nullptr, 0);
}

class Coalescer {
public:
	Coalescer()
	    : nslots_(env_int("NET2_COALESCE_SLOTS", 8, 1, kMaxSlots)),
	      window_(std::chrono::microseconds(
		  env_int("NET2_COALESCE_WINDOW_US", 20, 0, 100000))),
	      zerocopy_(env_int("NET2_COALESCE_ZEROCOPY", 1, 0, 1) != 0),
	      jobmode_(env_int("NET2_COALESCE_JOBMODE", 0, 0, 2)),
	      /* tests only: a small lane-form chunk runs the 4 GiB split on
	       * small jobs (NET2_COALESCE_JOB_CHUNK, in 128-byte units) */
	      job_chunk_(128u * (uint32_t)env_int("NET2_COALESCE_JOB_CHUNK",
		  1 << 24, 1, 1 << 24))
	{
		for (int i = nslots_ - 1; i >= 0; i--)
			free_.push_back(i);
	}

	int submit(int ordinal, const Request &r, int *hip_err);
	void stats(uint64_t *calls, uint64_t *launches) const
	{
		if (calls)
			*calls = calls_.load(std::memory_order_relaxed);
		if (launches)
			*launches = launches_.load(std::memory_order_relaxed);
	}

private:
	int grow_stage(Slot &s, size_t need, int ordinal);
	int launch_and_wait(Slot &s, int ordinal, int *hip_err);

	std::mutex mu_;
	std::condition_variable slot_cv_;	/* open batch / free slots */
	std::condition_variable lead_cv_;	/* leaders: inflight, full */
	Slot slot_[kMaxSlots];
	const int nslots_;
	const clk::duration window_;
	const bool zerocopy_;
	const int jobmode_;	/* 0 auto, 1 wave per job, 2 lane per job */
	const uint32_t job_chunk_;
	int open_ = -1;
	std::vector<int> free_;
	int inflight_ = 0;
	std::atomic<uint64_t> calls_{0}, launches_{0};
};

int Coalescer::grow_stage(Slot &s, size_t need, int ordinal)
{
	/* only for an empty open batch, with the device mutex held; device
	 * memory goes on `ordinal`, whatever the caller's current device */
	int prev = -1;
	(void)hipGetDevice(&prev);
	struct Restore {
		int dev;
		~Restore() { if (dev >= 0) (void)hipSetDevice(dev); }
	} restore = { prev };
	if (hipSetDevice(ordinal) != hipSuccess)
		return EIO;
	size_t cap = std::max(kInitialStage, need + need / 4);
	s.free_stage();
	uint8_t *h = nullptr, *d = nullptr;
	if (host_alloc(&h, cap, zerocopy_) != hipSuccess)
		return ENOMEM;
	if (zerocopy_) {
		if (hipHostGetDevicePointer((void **)&d, h, 0) != hipSuccess) {
			(void)hipHostFree(h);
			return ENOMEM;
		}
	} else if (hipMalloc((void **)&d, cap) != hipSuccess) {
		(void)hipHostFree(h);
		return ENOMEM;
	}
	s.h_stage = h;
	s.d_stage = d;
	s.cap = cap;
	return 0;
}

size_t iov_total(const struct iovec *iov, size_t n)
{
	size_t t = 0;
	for (size_t i = 0; i < n; i++)
		t += iov[i].iov_len;
	return t;
}

uint8_t *gather(uint8_t *dst, const struct iovec *iov, size_t n)
{
	for (size_t i = 0; i < n; i++) {
		if (iov[i].iov_len)
			memcpy(dst, iov[i].iov_base, iov[i].iov_len);
		dst += iov[i].iov_len;
	}
	return dst;
}

/* Bytes of a padded message of `len` bytes: 0x80, zeros, the 64-bit
 * (SHA-256) or 128-bit (SHA-384/512) big-endian bit count. */
size_t padded_len(size_t len, size_t blk)
{
	const size_t lenbytes = blk == 64 ? 8 : 16;
	return (len + 1 + lenbytes + blk - 1) / blk * blk;
}

/* Terminator, zero fill and bit count after `len` message bytes at p
 * (which starts the padded message of padded_len(len) bytes). */
void put_pad(uint8_t *p, size_t len, size_t blk, uint64_t bits)
{
	const size_t total = padded_len(len, blk);
	p[len] = 0x80;
	memset(p + len + 1, 0, total - len - 1);
	for (int i = 0; i < 8; i++)
		p[total - 1 - i] = (uint8_t)(bits >> (8 * i));
}

void key_block(uint8_t *p, const uint8_t *key, size_t keylen, size_t blk,
    uint8_t pad)
{
	for (size_t i = 0; i < blk; i++)
		p[i] = (uint8_t)((i < keylen ? key[i] : 0) ^ pad);
}

int Coalescer::submit(int ordinal, const Request &r, int *hip_err)
{
	const size_t blk = r.alg == 1 ? 64 : 128;
	const size_t msg = iov_total(r.iov, r.iovcnt);
	size_t body, aux;

	switch (r.kind) {
	case DIGEST:
		body = padded_len(msg, blk);
		aux = 0;
		break;
	case HMAC:
		if (r.keylen > blk)
			return EINVAL;
		body = padded_len(blk + msg, blk);
		aux = blk;
		break;
	case BLOCKS:
		if (msg % blk != 0 || r.state == nullptr)
			return EINVAL;
		body = msg;
		aux = 64;
		break;
	default:
		return EINVAL;
	}
	const size_t need = align64(body + aux);
	const size_t nblk = body / blk;
	/* the wave form walks a job in 64-block steps of a 32-bit block index:
	 * keep its last step below 2^32 (a job of 2^32 - 64 blocks is 256 GiB
	 * of SHA-256, 512 GiB of SHA-512) */
	if (nblk > UINT32_MAX - 64)
		return EINVAL;

	Job job;
	job.kind = r.kind;
	job.alg = r.alg;
	job.out = r.out;
	std::unique_lock<std::mutex> lk(mu_);
	int si;
	for (;;) {
		if (open_ < 0) {
			if (free_.empty()) {
				slot_cv_.wait(lk);
				continue;
			}
			open_ = free_.back();
			free_.pop_back();
			Slot &s = slot_[open_];
			s.jobs.clear();
			s.used = 0;
			s.full = false;
			s.opened = clk::now();
		}
		Slot &s = slot_[open_];
		const size_t hdr = (s.jobs.size() + 1) * sizeof(Net2Job);
		if (s.used + need + hdr <= s.cap && s.jobs.size() < kMaxJobs)
			break;
		if (s.jobs.empty()) {
			int rc = grow_stage(s, need + hdr, ordinal);
			if (rc != 0)
				return rc;
			continue;
		}
		/* no room: the leader launches it now; join the next batch */
		s.full = true;
		lead_cv_.notify_all();
		const int cur = open_;
		slot_cv_.wait(lk, [&]() { return open_ != cur; });
	}
	si = open_;
	Slot &s = slot_[si];
	const size_t off = s.used;
	s.used += need;
	s.jobs.push_back(&job);
	s.writers.fetch_add(1, std::memory_order_relaxed);
	const bool leader = s.jobs.size() == 1;
	if (!leader && s.used + 2 * 1024 > s.cap) {
		s.full = true;
		lead_cv_.notify_all();
	}
	lk.unlock();

	/* lay the job out in staging (no lock: the range is ours) */
	uint8_t *p = s.h_stage + off;
	job.desc.data = off;
	job.desc.aux = off + body;
	job.desc.nblk = (uint32_t)nblk;
	job.desc.flags = (uint32_t)r.alg;
	if (r.kind == DIGEST) {
		gather(p, r.iov, r.iovcnt);
		put_pad(p, msg, blk, (uint64_t)msg << 3);
	} else if (r.kind == HMAC) {
		key_block(p, r.key, r.keylen, blk, 0x36);
		gather(p + blk, r.iov, r.iovcnt);
		put_pad(p, blk + msg, blk, (uint64_t)(blk + msg) << 3);
		key_block(p + body, r.key, r.keylen, blk, 0x5c);
		job.desc.flags |= NET2_JOB_HMAC;
	} else {
		gather(p, r.iov, r.iovcnt);
		memcpy(p + body, r.state, blk == 64 ? 32 : 64);
		job.desc.flags |= NET2_JOB_STATE;
	}
	s.writers.fetch_sub(1, std::memory_order_release);

	if (!leader) {
		/* a short spin, then sleep until the leader posts our result */
		for (int i = 0; i < 256 && !job.done.load(std::memory_order_acquire); i++)
			__builtin_ia32_pause();
		while (!job.done.load(std::memory_order_acquire))
			futex_wait(&job.done, 0);
		if (job.rc == EIO && hip_err != nullptr)
			*hip_err = job.hip;
		return job.rc;
	}

	/* leader: launch when the device is idle, the batch full, or the
	 * window over */
	lk.lock();
	lead_cv_.wait_until(lk, s.opened + window_, [&]() {
		return inflight_ == 0 || s.full;
	});
	if (open_ == si) {
		open_ = -1;		/* later callers open the next batch */
		slot_cv_.notify_all();
	}
	inflight_++;
	lk.unlock();
	/* every reservation is in (the batch is closed); wait for the copies */
	while (s.writers.load(std::memory_order_acquire) != 0)
		__builtin_ia32_pause();

	int herr = 0;
	const int rc = launch_and_wait(s, ordinal, &herr);
	launches_.fetch_add(1, std::memory_order_relaxed);
	calls_.fetch_add(s.jobs.size(), std::memory_order_relaxed);
	if (rc == EIO && hip_err != nullptr)
		*hip_err = herr;
	for (Job *jp : s.jobs) {
		if (jp == &job)
			continue;
		jp->rc = rc;
		jp->hip = herr;
		std::atomic<int> *w = &jp->done;
		w->store(1, std::memory_order_release);
		futex_wake(w);		/* jp may be gone now; the address is inert */
	}

	/* the slot is still ours (not on free_): shrink outside the lock, once
	 * oversized staging serves a batch that needs little of it */
	if (s.cap > kRetainStage && s.used * 4 < s.cap)
		s.free_stage();
	lk.lock();
	s.jobs.clear();
	inflight_--;
	free_.push_back(si);
	lead_cv_.notify_all();
	slot_cv_.notify_all();
	return rc;
}

void store_be32(uint8_t *p, uint32_t v)
{
	p[0] = (uint8_t)(v >> 24);
	p[1] = (uint8_t)(v >> 16);
	p[2] = (uint8_t)(v >> 8);
	p[3] = (uint8_t)v;
}

/* Raw state words -> the caller's output (digest bytes as SHA*Final
 * stores them, src/sha2.c:553-557 / :847-850 / :905-908, or the state). */
void deliver(const Job &j, const uint8_t *raw)
{
	if (j.kind == BLOCKS) {
		memcpy(j.out, raw, j.alg == 1 ? 32 : 64);
		return;
	}
	if (j.alg == 1) {
		uint32_t w[8];
		memcpy(w, raw, sizeof(w));
		for (int i = 0; i < 8; i++)
			store_be32(j.out + 4 * i, w[i]);
		return;
	}
	uint64_t w[8];
	memcpy(w, raw, sizeof(w));
	for (int i = 0; i < (j.alg == 2 ? 6 : 8); i++) {
		store_be32(j.out + 8 * i, (uint32_t)(w[i] >> 32));
		store_be32(j.out + 8 * i + 4, (uint32_t)w[i]);
	}
}

int Coalescer::launch_and_wait(Slot &s, int ordinal, int *hip_err)
{
	int prev = -1;
	(void)hipGetDevice(&prev);
	struct Restore {
		int dev;
		~Restore() { if (dev >= 0) (void)hipSetDevice(dev); }
	} restore = { prev };
	hipError_t e;
#define CO_TRY(expr)                                                         \
	do {                                                                 \
		if ((e = (expr)) != hipSuccess)                              \
			goto fail;                                           \
	} while (0)

	std::vector<Job *> &jobs = s.jobs;
	const size_t n = jobs.size();
	size_t hdr_off, n256;
	uint32_t waves, target;
	int wave;
	const uint8_t *stage;
	uint8_t *d_out;
	uint32_t *d_done;

	CO_TRY(hipSetDevice(ordinal));
	/* each resource is created once and kept; a failed creation leaves its
	 * field null, so the next batch retries just that one */
	if (s.stream == nullptr)
		CO_TRY(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
	if (s.ev == nullptr)
		CO_TRY(hipEventCreateWithFlags(&s.ev, hipEventDisableTiming));
	if (s.h_done == nullptr) {
		CO_TRY(hipHostMalloc((void **)&s.h_done, 64,
		    hipHostMallocMapped | hipHostMallocCoherent));
		*s.h_done = 0;
		s.done_base = 0;
	}
	if (s.cap_jobs < n) {
		/* results are written by the kernel straight into coherent
		 * host memory: no copy back, no wait for one */
		const size_t want = std::max<size_t>(n + n / 2, 256);
		s.free_out();
		CO_TRY(hipHostMalloc((void **)&s.h_out, want * 64,
		    hipHostMallocMapped | hipHostMallocCoherent));
		s.cap_jobs = want;
	}
	CO_TRY(hipHostGetDevicePointer((void **)&d_out, s.h_out, 0));
	CO_TRY(hipHostGetDevicePointer((void **)&d_done, s.h_done, 0));
	/* In a lane-form batch, jobs of kWaveBlocks or more first (each takes
	 * a wave of its own in a launch of their own -- a lane would run one
	 * alone for a long time); then SHA-256 jobs, then SHA-384/512 (the
	 * launches take each family as one run), longest first within each,
	 * so a wave's lanes share their trip count as far as possible */
	wave = jobmode_ == 1 || (jobmode_ == 0 && n <= kWaveJobsMax);
	std::sort(jobs.begin(), jobs.end(), [wave, this](const Job *a,
	    const Job *b) {
		const int la = !wave && jobmode_ == 0 &&
		    a->desc.nblk >= kWaveBlocks;
		const int lb = !wave && jobmode_ == 0 &&
		    b->desc.nblk >= kWaveBlocks;
		if (la != lb)
			return la > lb;
		const int fa = a->alg != 1, fb = b->alg != 1;
		if (fa != fb)
			return fa < fb;
		return a->desc.nblk > b->desc.nblk;
	});
	hdr_off = align64(s.used);
	n256 = 0;
	for (size_t k = 0; k < n; k++) {
		memcpy(s.h_stage + hdr_off + k * sizeof(Net2Job), &jobs[k]->desc,
		    sizeof(Net2Job));
		n256 += jobs[k]->alg == 1;
	}
	if (!zerocopy_)
		CO_TRY(hipMemcpyAsync(s.d_stage, s.h_stage,
		    hdr_off + n * sizeof(Net2Job), hipMemcpyHostToDevice,
		    s.stream));
	stage = s.d_stage;
	/* few jobs: a wave each (lower latency, the GPU is idle anyway);
	 * many: a lane each -- except the long jobs at the front, which take
	 * a wave each in a launch of their own, so one long request does not
	 * switch a whole batch of small ones to the wave form */
	if (wave) {
		waves = (uint32_t)n;
		target = s.done_base + waves;
		CO_TRY(net2_launch_jobs(stage,
		    reinterpret_cast<const Net2Job *>(stage + hdr_off),
		    (uint32_t)n256, (uint32_t)(n - n256), d_out, d_done, 1,
		    s.stream, job_chunk_));
	} else {
		size_t nl = 0, nl256 = 0;
		if (jobmode_ == 0)
			for (; nl < n && jobs[nl]->desc.nblk >= kWaveBlocks; nl++)
				nl256 += jobs[nl]->alg == 1;
		const size_t ns256 = n256 - nl256, ns512 = n - nl - ns256;
		waves = (uint32_t)(nl + (ns256 + 63) / 64 + (ns512 + 63) / 64);
		target = s.done_base + waves;
		const Net2Job *hj =
		    reinterpret_cast<const Net2Job *>(stage + hdr_off);
		if (nl > 0)
			CO_TRY(net2_launch_jobs(stage, hj, (uint32_t)nl256,
			    (uint32_t)(nl - nl256), d_out, d_done, 1, s.stream,
			    job_chunk_));
		if (nl < n)
			CO_TRY(net2_launch_jobs(stage, hj + nl, (uint32_t)ns256,
			    (uint32_t)ns512, d_out + 64 * nl, d_done, 0, s.stream,
			    job_chunk_));
	}
	CO_TRY(hipEventRecord(s.ev, s.stream));
	{
		/*
		 * Done when every wave has counted itself in (each stores its
		 * results first, then adds 1 with system-scope release order).
		 * A small batch takes tens of microseconds: poll the host word
		 * (no runtime call, no end-of-kernel latency); after a few
		 * milliseconds fall back to the event, which also reports a
		 * kernel that failed.
		 */
		const clk::time_point t0 = clk::now();
		bool ok = false;
		for (unsigned i = 1;; i++) {
			if (__atomic_load_n(s.h_done, __ATOMIC_ACQUIRE) == target) {
				ok = true;
				break;
			}
			if ((i & 255) == 0 &&
			    clk::now() - t0 > std::chrono::milliseconds(5))
				break;
			__builtin_ia32_pause();
		}
		if (!ok) {
			CO_TRY(hipEventSynchronize(s.ev));
			if (__atomic_load_n(s.h_done, __ATOMIC_ACQUIRE) != target) {
				e = hipErrorLaunchFailure;
				goto fail;
			}
		}
		s.done_base = target;
	}
	for (size_t k = 0; k < n; k++)
		deliver(*jobs[k], s.h_out + 64 * k);
	return 0;
fail:
	if (hip_err != nullptr)
		*hip_err = (int)e;
	(void)hipGetLastError();
	/* the counter may be anywhere now: resynchronise it */
	if (s.stream != nullptr && hipStreamSynchronize(s.stream) == hipSuccess &&
	    s.h_done != nullptr)
		s.done_base = __atomic_load_n(s.h_done, __ATOMIC_ACQUIRE);
	return e == hipErrorOutOfMemory ? ENOMEM : EIO;
#undef CO_TRY
}

std::mutex g_mu;
std::vector<std::unique_ptr<Coalescer>> g_co;

Coalescer *coalescer(size_t idx)
{
	std::lock_guard<std::mutex> g(g_mu);
	if (g_co.size() <= idx)
		g_co.resize(idx + 1);
	if (!g_co[idx])
		g_co[idx].reset(new Coalescer());
	return g_co[idx].get();
}

}	/* namespace */

void stats(size_t idx, uint64_t *calls, uint64_t *launches)
{
	Coalescer *c = nullptr;
	{
		std::lock_guard<std::mutex> g(g_mu);
		if (idx < g_co.size())
			c = g_co[idx].get();
	}
	if (c != nullptr) {
		c->stats(calls, launches);
		return;
	}
	if (calls)
		*calls = 0;
	if (launches)
		*launches = 0;
}

int submit(size_t idx, int ordinal, const Request &r, int *hip_err)
{
	if (r.alg < 1 || r.alg > 3 || (r.iovcnt > 0 && r.iov == nullptr) ||
	    r.out == nullptr)
		return EINVAL;
	return coalescer(idx)->submit(ordinal, r, hip_err);
}

}	/* namespace net2co */
