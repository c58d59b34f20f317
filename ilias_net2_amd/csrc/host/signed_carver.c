/*
 * signed_carver.c -- the hashing and signing steps of src/signed_carver.c,
 * batched per workq tick (include/net2/signed_carver.h).
 *
 * One tick: (1) every payload of the tick, from hash requests, new
 * carvers and combiner checks alike, is hashed once -- all payloads of one
 * hash algorithm in one net2_sha2_batch call (the reference hashes each
 * payload once per sign context, src/signed_carver.c:407-411 ->
 * signature.n2t:92); (2) the work after the hash -- the hash requests'
 * callbacks (the caller's own ECDSA, e.g. the reference's sign.c),
 * num_signatures signatures per carver (:407-432), one verification per
 * check (:305-319) -- is spread over host threads.
 */
#include "../../../include/net2/signed_carver.h"
#include "../../../include/net2/hash.h"
#include "signature_int.h"

#include <errno.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#define NET2_EXPORT __attribute__((visibility("default")))

/* ---- one tick -------------------------------------------------------- */

/* One payload to hash: where its digest goes. */
struct payload_ref {
	const struct iovec	*iov;
	size_t			 iovcnt;
	int			 alg;		/* 1..3, or < 0: not hashed */
	uint8_t			*digest;	/* 64 bytes */
	int			*rc;		/* set on a hash failure */
};

static size_t
iov_len(const struct iovec *iov, size_t n)
{
	size_t t = 0;

	for (size_t i = 0; i < n; i++)
		t += iov[i].iov_len;
	return t;
}

/*
 * A few long payloads: one net2_hashctx_hashiov per payload, submitted from
 * as many threads at once, so the request coalescer runs them as one batch
 * in its wave-per-message form (the 64 lanes expand a message's schedules
 * in parallel; a lone 64 KiB SHA-512 payload: ~2.0 ms, against ~3.6 ms as
 * one lane of a net2_sha2_batch, profiles/round4/latency_long.jsonl).
 */
#define NET2_SC_FEW 16			/* the coalescer's wave-form batch */
#define NET2_SC_LONG_BYTES 8192		/* mean payload above which it pays */

/*
 * Helper threads of the tick, started once and kept: the hash requests of a
 * few long payloads (hash_few_long) and the work after the hash (run_jobs)
 * run on them instead of on threads created and joined every tick.  A
 * batch's tasks go on one queue that every worker -- and the submitting
 * thread, while it waits for its batch -- takes from, so concurrent ticks
 * share the workers and none waits on a task nobody runs.  The workers are
 * detached and live as long as the process.
 */
#define NET2_SC_MAXTHREADS 64

struct sc_batch {
	size_t		left;		/* tasks not finished */
	pthread_cond_t	done;
};

struct sc_task {
	void		*(*fn)(void *);
	void		*arg;
	struct sc_batch	*b;
	int		 dev;		/* the submitter's device index */
};

static struct {
	pthread_mutex_t	mu;
	pthread_cond_t	work;
	struct sc_task	*q;		/* ring of qcap tasks */
	size_t		qcap, qhead, qlen;
	int		nworkers;
} g_pool = { PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER, NULL,
    0, 0, 0, 0 };

/* the next queued task, under g_pool.mu; 0 if none */
static int
pool_pop(struct sc_task *t)
{
	if (g_pool.qlen == 0)
		return 0;
	*t = g_pool.q[g_pool.qhead];
	g_pool.qhead = (g_pool.qhead + 1) % g_pool.qcap;
	g_pool.qlen--;
	return 1;
}

/*
 * run t outside the lock, then count it done (lock held on entry/exit).  The
 * task runs on its submitter's GPU (net2_sha2_set_device): a helper thread
 * has no device of its own, and one that helps another tick must not hash
 * that tick's payloads on its own device.
 */
static void
pool_run(struct sc_task *t)
{
	int own = -1, prev = -1, set = 0;

	pthread_mutex_unlock(&g_pool.mu);
	if (t->dev >= 0 && net2_sha2_get_device(&own) == 0 && own != t->dev)
		set = net2_sha2_set_device(t->dev, &prev) == 0;
	t->fn(t->arg);
	if (set) {
		/* back to this thread's own device (and its HIP device: the
		 * selection moved it), then to its own selection */
		(void)net2_sha2_set_device(prev >= 0 ? prev : own, NULL);
		if (prev < 0)
			(void)net2_sha2_set_device(-1, NULL);
	}
	pthread_mutex_lock(&g_pool.mu);
	if (--t->b->left == 0)
		pthread_cond_broadcast(&t->b->done);
}

static void *
pool_worker(void *unused)
{
	struct sc_task t;

	(void)unused;
	pthread_setname_np(pthread_self(), "net2-sc");
	pthread_mutex_lock(&g_pool.mu);
	for (;;) {
		while (!pool_pop(&t))
			pthread_cond_wait(&g_pool.work, &g_pool.mu);
		pool_run(&t);
	}
	return NULL;
}

/*
 * fn(args[k]) for k < n, on the calling thread and up to nthreads - 1
 * helpers; returns when all are done.  Tasks that cannot be queued (no
 * memory) or find no helper run on the calling thread.
 */
static void
pool_run_batch(void *(*fn)(void *), void **args, size_t n, int nthreads)
{
	struct sc_batch b;
	struct sc_task t;
	size_t k;
	int dev = -1;

	if (n == 0)
		return;
	if (n == 1 || nthreads <= 1) {
		for (k = 0; k < n; k++)
			fn(args[k]);
		return;
	}
	b.left = n - 1;
	if (net2_sha2_get_device(&dev) != 0)
		dev = -1;
	pthread_cond_init(&b.done, NULL);
	pthread_mutex_lock(&g_pool.mu);
	/* room for this batch's tasks on the ring */
	if (g_pool.qcap < g_pool.qlen + n) {
		size_t cap = 2 * (g_pool.qlen + n);
		struct sc_task *q = malloc(cap * sizeof(*q));
		if (q != NULL) {
			for (k = 0; k < g_pool.qlen; k++)
				q[k] = g_pool.q[(g_pool.qhead + k) % g_pool.qcap];
			free(g_pool.q);
			g_pool.q = q;
			g_pool.qcap = cap;
			g_pool.qhead = 0;
		}
	}
	if (g_pool.qcap < g_pool.qlen + n) {
		pthread_mutex_unlock(&g_pool.mu);
		pthread_cond_destroy(&b.done);
		for (k = 0; k < n; k++)
			fn(args[k]);
		return;
	}
	while (g_pool.nworkers < nthreads - 1 &&
	    g_pool.nworkers < NET2_SC_MAXTHREADS - 1) {
		pthread_t tid;
		if (pthread_create(&tid, NULL, pool_worker, NULL) != 0)
			break;
		pthread_detach(tid);
		g_pool.nworkers++;
	}
	for (k = 1; k < n; k++) {
		g_pool.q[(g_pool.qhead + g_pool.qlen) % g_pool.qcap] =
		    (struct sc_task){ fn, args[k], &b, dev };
		g_pool.qlen++;
	}
	pthread_cond_broadcast(&g_pool.work);
	pthread_mutex_unlock(&g_pool.mu);
	fn(args[0]);
	pthread_mutex_lock(&g_pool.mu);
	/* help with whatever is queued until this batch is done */
	while (b.left > 0) {
		if (pool_pop(&t))
			pool_run(&t);
		else
			pthread_cond_wait(&b.done, &g_pool.mu);
	}
	pthread_mutex_unlock(&g_pool.mu);
	pthread_cond_destroy(&b.done);
}

struct one_hash {
	const struct payload_ref *p;
	int alg, rc;
};

static void *
one_hash_run(void *arg)
{
	struct one_hash *o = arg;

	o->rc = net2_hashctx_hashiov(o->alg, NULL, 0, o->p->iov, o->p->iovcnt,
	    o->p->digest, 64);
	return NULL;
}

static int
hash_few_long(struct payload_ref *p, size_t np, int alg)
{
	struct one_hash job[NET2_SC_FEW];
	void *args[NET2_SC_FEW];
	size_t m = 0;
	int rc = 0;

	for (size_t i = 0; i < np; i++)
		if (p[i].alg == alg) {
			job[m] = (struct one_hash){ &p[i], alg, 0 };
			args[m] = &job[m];
			m++;
		}
	/* all at once, so the coalescer batches them */
	pool_run_batch(one_hash_run, args, m, (int)m);
	for (size_t k = 0; k < m; k++)
		if (job[k].rc != 0) {
			if (*job[k].p->rc == 0)
				*job[k].p->rc = job[k].rc;
			rc = rc ? rc : job[k].rc;
		}
	return rc;
}

/*
 * Hash every payload of algorithm alg in one net2_sha2_batch call.
 * Single-segment payloads are passed in place, as offsets from the lowest
 * payload address; multi-segment ones are gathered first.
 */
static int
hash_group(struct payload_ref *p, size_t np, int alg)
{
	size_t m = 0, gathered = 0;
	uintptr_t lo = UINTPTR_MAX;
	uint64_t *offs = NULL;
	uint32_t *lens = NULL;
	uint8_t *dig = NULL, *gbuf = NULL, *at;
	const int hl = net2_hash_gethashlen(alg);
	int rc = 0;

	for (size_t i = 0; i < np; i++) {
		if (p[i].alg != alg)
			continue;
		m++;
		if (p[i].iovcnt > 1)
			gathered += iov_len(p[i].iov, p[i].iovcnt);
	}
	if (m == 0)
		return 0;
	if (m <= NET2_SC_FEW) {
		size_t total = 0;
		for (size_t i = 0; i < np; i++)
			if (p[i].alg == alg)
				total += iov_len(p[i].iov, p[i].iovcnt);
		if (total >= m * (size_t)NET2_SC_LONG_BYTES)
			return hash_few_long(p, np, alg);
	}
	offs = malloc(m * sizeof(*offs));
	lens = malloc(m * sizeof(*lens));
	dig = malloc(m * (size_t)hl);
	gbuf = malloc(gathered ? gathered : 1);
	if (offs == NULL || lens == NULL || dig == NULL || gbuf == NULL) {
		rc = ENOMEM;
		goto out;
	}
	/* the address of every payload's bytes, then offsets from the lowest */
	at = gbuf;
	m = 0;
	for (size_t i = 0; i < np; i++) {
		if (p[i].alg != alg)
			continue;
		const size_t len = iov_len(p[i].iov, p[i].iovcnt);
		uintptr_t a;
		if (len > UINT32_MAX) {
			rc = EINVAL;
			goto out;
		}
		if (p[i].iovcnt > 1) {
			a = (uintptr_t)at;
			for (size_t k = 0; k < p[i].iovcnt; k++) {
				if (p[i].iov[k].iov_len)
					memcpy(at, p[i].iov[k].iov_base,
					    p[i].iov[k].iov_len);
				at += p[i].iov[k].iov_len;
			}
		} else {
			a = p[i].iovcnt == 1 ? (uintptr_t)p[i].iov[0].iov_base :
			    (uintptr_t)gbuf;
		}
		offs[m] = a;
		lens[m] = (uint32_t)len;
		if (a < lo)
			lo = a;
		m++;
	}
	for (size_t k = 0; k < m; k++)
		offs[k] -= lo;
	rc = net2_sha2_batch(alg, (const void *)lo, offs, lens, 0, 0, m, dig,
	    0);
	if (rc == 0) {
		m = 0;
		for (size_t i = 0; i < np; i++)
			if (p[i].alg == alg)
				memcpy(p[i].digest, dig + (m++) * (size_t)hl,
				    (size_t)hl);
	}
out:
	if (rc != 0)
		for (size_t i = 0; i < np; i++)
			if (p[i].alg == alg && *p[i].rc == 0)
				*p[i].rc = rc;
	free(offs);
	free(lens);
	free(dig);
	free(gbuf);
	return rc;
}

/* Jobs after the hash: job j < nsig_jobs signs, the next nv validate, the
 * last nh run the hash requests' callbacks. */
struct ecdsa_plan {
	struct net2_sc_hash_req		**hreq;
	size_t				 nh;
	struct net2_sc_sign_req		*sreq;
	size_t				 ns;
	struct net2_sc_validate_req	*vreq;
	size_t				 nv;
	const uint8_t			*sdig;	/* ns x 64 */
	const uint8_t			*vdig;	/* nv x 64 */
	const int			*valg;	/* hash row per check, < 0 bad */
	const size_t			*sjob;	/* prefix sums of num_signatures */
	size_t				 nsig_jobs, njobs;
};

struct ecdsa_slice {
	const struct ecdsa_plan	*pl;
	size_t			 lo, hi;
};

/* request index of signature job j (binary search over the prefix sums) */
static size_t
sign_req_of(const struct ecdsa_plan *pl, size_t j)
{
	size_t a = 0, b = pl->ns;

	while (b - a > 1) {
		size_t c = (a + b) / 2;
		if (pl->sjob[c] <= j)
			a = c;
		else
			b = c;
	}
	return a;
}

static void *
ecdsa_run(void *arg)
{
	const struct ecdsa_slice *sl = arg;
	const struct ecdsa_plan *pl = sl->pl;

	for (size_t j = sl->lo; j < sl->hi; j++) {
		if (j < pl->nsig_jobs) {
			const size_t r = sign_req_of(pl, j);
			struct net2_sc_sign_req *q = &pl->sreq[r];
			const size_t k = j - pl->sjob[r];
			/* a sibling signature may have failed already */
			if (__atomic_load_n(&q->rc, __ATOMIC_RELAXED) != 0)
				continue;
			int rc = sign_digest(&q->out[k], pl->sdig + 64 * r,
			    (size_t)net2_hash_gethashlen(q->hash_alg),
			    net2_hash_getname(q->hash_alg), q->signatures[k]);
			if (rc != 0)
				__atomic_store_n(&q->rc, rc, __ATOMIC_RELAXED);
			continue;
		}
		if (j >= pl->nsig_jobs + pl->nv) {
			struct net2_sc_hash_req *h =
			    pl->hreq[j - pl->nsig_jobs - pl->nv];
			if (h->done != NULL)
				h->done(h, h->arg);
			continue;
		}
		const size_t v = j - pl->nsig_jobs;
		struct net2_sc_validate_req *q = &pl->vreq[v];
		if (pl->valg[v] < 0 || q->result != 0)
			continue;
		if (strcmp(net2x_signctx_name(q->sctx), q->sig->sign_alg) != 0) {
			q->result = EIO;	/* signature.n2t:155-158 -> :333-336 */
			continue;
		}
		q->result = net2x_signctx_validate(q->sctx, q->sig->data,
		    q->sig->datalen, pl->vdig + 64 * v,
		    (size_t)net2_hash_gethashlen(pl->valg[v])) == 1 ? 0 : EINVAL;
	}
	return NULL;
}

static void
run_jobs(const struct ecdsa_plan *pl, int nthreads)
{
	struct ecdsa_slice sl[NET2_SC_MAXTHREADS];
	void *args[NET2_SC_MAXTHREADS];
	int t;

	if (nthreads <= 0) {
		long c = sysconf(_SC_NPROCESSORS_ONLN);
		nthreads = c > 0 ? (int)c : 1;
	}
	if (nthreads > NET2_SC_MAXTHREADS)
		nthreads = NET2_SC_MAXTHREADS;
	if ((size_t)nthreads > pl->njobs)
		nthreads = pl->njobs ? (int)pl->njobs : 1;
	for (t = 0; t < nthreads; t++) {
		sl[t].pl = pl;
		sl[t].lo = pl->njobs * t / nthreads;
		sl[t].hi = pl->njobs * (t + 1) / nthreads;
		args[t] = &sl[t];
	}
	pool_run_batch(ecdsa_run, args, (size_t)nthreads, nthreads);
}

/* validate_prologue of signature.c (signature.n2t:133-145): hash row of a
 * decoded signature, or -1 when it cannot be validated */
static int
check_alg(const struct net2_sc_validate_req *q)
{
	int alg;

	if (q->sig == NULL || q->sctx == NULL || q->sig->data == NULL ||
	    q->sig->hash_alg == NULL || q->sig->sign_alg == NULL ||
	    (q->payload == NULL && q->iovcnt > 0))
		return -1;
	if ((alg = net2_hash_findname(q->sig->hash_alg)) < 0 ||
	    net2_hash_getkeylen(alg) != 0 || net2_hash_gethashlen(alg) <= 0)
		return -1;
	return alg;
}

/* a hash request's row: an unkeyed registry row with a digest */
static int
hash_req_ok(const struct net2_sc_hash_req *h)
{
	return !(h->payload == NULL && h->iovcnt > 0) &&
	    net2_hash_getname(h->hash_alg) != NULL &&
	    net2_hash_gethashlen(h->hash_alg) > 0 &&
	    net2_hash_getkeylen(h->hash_alg) == 0;
}

static int
tick(struct net2_sc_hash_req **hreq, size_t nh,
    struct net2_sc_sign_req *sreq, size_t ns,
    struct net2_sc_validate_req *vreq, size_t nv, int nthreads)
{
	struct payload_ref *p = NULL;
	uint8_t *sdig = NULL, *vdig = NULL;
	int *valg = NULL, rc = 0;
	size_t *sjob = NULL, np = 0;
	struct ecdsa_plan pl;

	if (nh + ns + nv == 0)
		return 0;
	for (size_t i = 0; i < nh; i++) {
		hreq[i]->rc = hash_req_ok(hreq[i]) ? 0 : EINVAL;
		hreq[i]->digestlen = 0;
	}
	p = calloc(nh + ns + nv, sizeof(*p));
	sdig = malloc(ns * 64 + 1);
	vdig = malloc(nv * 64 + 1);
	valg = malloc((nv + 1) * sizeof(*valg));
	sjob = malloc((ns + 1) * sizeof(*sjob));
	if (p == NULL || sdig == NULL || vdig == NULL || valg == NULL ||
	    sjob == NULL) {
		rc = ENOMEM;
		for (size_t i = 0; i < ns; i++)
			sreq[i].rc = ENOMEM;
		for (size_t i = 0; i < nv; i++)
			vreq[i].result = EIO;
		/* every callback runs once, whatever the outcome */
		for (size_t i = 0; i < nh; i++) {
			hreq[i]->rc = ENOMEM;
			if (hreq[i]->done != NULL)
				hreq[i]->done(hreq[i], hreq[i]->arg);
		}
		goto out;
	}
	/* requests -> payloads to hash */
	for (size_t i = 0; i < nh; i++) {
		struct net2_sc_hash_req *h = hreq[i];
		p[np++] = (struct payload_ref){ h->payload, h->iovcnt,
		    h->rc == 0 ? h->hash_alg : -1, h->digest, &h->rc };
	}
	sjob[0] = 0;
	for (size_t i = 0; i < ns; i++) {
		struct net2_sc_sign_req *q = &sreq[i];
		q->rc = 0;
		if (q->out == NULL || (q->num_signatures > 0 &&
		    q->signatures == NULL) || (q->payload == NULL &&
		    q->iovcnt > 0) || net2_hash_getname(q->hash_alg) == NULL ||
		    net2_hash_gethashlen(q->hash_alg) <= 0 ||
		    net2_hash_getkeylen(q->hash_alg) != 0)
			q->rc = EINVAL;		/* signature.n2t:69-72 */
		else
			memset(q->out, 0, q->num_signatures * sizeof(*q->out));
		sjob[i + 1] = sjob[i] + (q->rc == 0 ? q->num_signatures : 0);
		p[np++] = (struct payload_ref){ q->payload, q->iovcnt,
		    q->rc == 0 ? q->hash_alg : -1, sdig + 64 * i, &q->rc };
	}
	for (size_t i = 0; i < nv; i++) {
		struct net2_sc_validate_req *q = &vreq[i];
		valg[i] = check_alg(q);
		q->result = valg[i] < 0 ? EIO : 0;
		p[np++] = (struct payload_ref){ q->payload, q->iovcnt, valg[i],
		    vdig + 64 * i, &q->result };
	}
	/* one GPU batch per hash algorithm; a group's failure is in the rc /
	 * result of each of its requests (hash_group), so the others go on */
	for (int alg = NET2_HASH_SHA256; alg <= NET2_HASH_SHA512; alg++)
		(void)hash_group(p, np, alg);
	for (size_t i = 0; i < nv; i++)
		if (vreq[i].result != 0) {
			vreq[i].result = EIO;	/* hash failure: :333-336 */
			valg[i] = -1;
		}
	for (size_t i = 0; i < nh; i++)
		if (hreq[i]->rc == 0)
			hreq[i]->digestlen =
			    (uint32_t)net2_hash_gethashlen(hreq[i]->hash_alg);
	/* the callbacks and the ECDSA work on host threads */
	pl.hreq = hreq;
	pl.nh = nh;
	pl.sreq = sreq;
	pl.ns = ns;
	pl.vreq = vreq;
	pl.nv = nv;
	pl.sdig = sdig;
	pl.vdig = vdig;
	pl.valg = valg;
	pl.sjob = sjob;
	pl.nsig_jobs = sjob[ns];
	pl.njobs = sjob[ns] + nv + nh;
	/* the hash requests' part of the tick's outcome, taken now: their rc
	 * is final once hashing is done, and a callback may free or reuse its
	 * request */
	int h_all = 1, h_first = 0;
	for (size_t i = 0; i < nh && h_all; i++) {
		h_all = hreq[i]->rc != 0;
		h_first = h_first ? h_first : hreq[i]->rc;
	}
	if (pl.njobs > 0)
		run_jobs(&pl, nthreads);
	/* a carver whose signing failed keeps none of its signatures */
	for (size_t i = 0; i < ns; i++)
		if (sreq[i].rc != 0 && sreq[i].out != NULL &&
		    sreq[i].rc != EINVAL)
			for (uint32_t k = 0; k < sreq[i].num_signatures; k++)
				net2x_signature_deinit(&sreq[i].out[k]);
	/* the tick failed as a whole only if every request did (a validation
	 * that ran and found the signature invalid, EINVAL, is an outcome, not
	 * a failure); then it returns the first request's error, which every
	 * request carries too.  Otherwise 0, and the per-request rc / result
	 * values are the outcome. */
	{
		int all = h_all, first = h_first;
		for (size_t i = 0; i < ns && all; i++) {
			all = sreq[i].rc != 0;
			first = first ? first : sreq[i].rc;
		}
		for (size_t i = 0; i < nv && all; i++) {
			all = vreq[i].result == EIO;
			first = first ? first : vreq[i].result;
		}
		if (all)
			rc = first;
	}
out:
	free(p);
	free(sdig);
	free(vdig);
	free(valg);
	free(sjob);
	return rc;
}

NET2_EXPORT int
net2_sc_hash_tick(struct net2_sc_hash_req *reqs, size_t n, int nthreads)
{
	struct net2_sc_hash_req **hp;
	int rc;

	if (n > 0 && reqs == NULL)
		return EINVAL;
	if (n == 0)
		return 0;
	if ((hp = malloc(n * sizeof(*hp))) == NULL) {
		for (size_t i = 0; i < n; i++) {
			reqs[i].rc = ENOMEM;
			reqs[i].digestlen = 0;
			if (reqs[i].done != NULL)
				reqs[i].done(&reqs[i], reqs[i].arg);
		}
		return ENOMEM;
	}
	for (size_t i = 0; i < n; i++)
		hp[i] = &reqs[i];
	rc = tick(hp, n, NULL, 0, NULL, 0, nthreads);
	free(hp);
	return rc;
}

NET2_EXPORT int
net2_signed_carver_sign_tick(struct net2_sc_sign_req *reqs, size_t n,
    int nthreads)
{
	if (n > 0 && reqs == NULL)
		return EINVAL;
	return tick(NULL, 0, reqs, n, NULL, 0, nthreads);
}

NET2_EXPORT int
net2_signed_combiner_validate_tick(struct net2_sc_validate_req *reqs,
    size_t n, int nthreads)
{
	if (n > 0 && reqs == NULL)
		return EINVAL;
	return tick(NULL, 0, NULL, 0, reqs, n, nthreads);
}

/* ---- the collector ---------------------------------------------------- */

struct net2_sc_collector {
	pthread_mutex_t			 mu;
	int				 nthreads;
	struct net2_sc_hash_req		**hash;
	size_t				 nhash, caphash;
	struct net2_sc_sign_req		**sign;
	size_t				 nsign, capsign;
	struct net2_sc_validate_req	**val;
	size_t				 nval, capval;
};

NET2_EXPORT struct net2_sc_collector *
net2_sc_collector_new(int nthreads)
{
	struct net2_sc_collector *c = calloc(1, sizeof(*c));

	if (c == NULL)
		return NULL;
	if (pthread_mutex_init(&c->mu, NULL) != 0) {
		free(c);
		return NULL;
	}
	c->nthreads = nthreads;
	return c;
}

NET2_EXPORT void
net2_sc_collector_free(struct net2_sc_collector *c)
{
	if (c == NULL)
		return;
	pthread_mutex_destroy(&c->mu);
	free(c->hash);
	free(c->sign);
	free(c->val);
	free(c);
}

static int
push(void ***arr, size_t *n, size_t *cap, void *item)
{
	if (*n == *cap) {
		size_t nc = *cap ? 2 * *cap : 64;
		void **na = realloc(*arr, nc * sizeof(*na));
		if (na == NULL)
			return ENOMEM;
		*arr = na;
		*cap = nc;
	}
	(*arr)[(*n)++] = item;
	return 0;
}

NET2_EXPORT int
net2_sc_collector_add_hash(struct net2_sc_collector *c,
    struct net2_sc_hash_req *r)
{
	int rc;

	if (c == NULL || r == NULL)
		return EINVAL;
	pthread_mutex_lock(&c->mu);
	rc = push((void ***)&c->hash, &c->nhash, &c->caphash, r);
	pthread_mutex_unlock(&c->mu);
	return rc;
}

NET2_EXPORT int
net2_sc_collector_add_sign(struct net2_sc_collector *c,
    struct net2_sc_sign_req *r)
{
	int rc;

	if (c == NULL || r == NULL)
		return EINVAL;
	pthread_mutex_lock(&c->mu);
	rc = push((void ***)&c->sign, &c->nsign, &c->capsign, r);
	pthread_mutex_unlock(&c->mu);
	return rc;
}

NET2_EXPORT int
net2_sc_collector_add_validate(struct net2_sc_collector *c,
    struct net2_sc_validate_req *r)
{
	int rc;

	if (c == NULL || r == NULL)
		return EINVAL;
	pthread_mutex_lock(&c->mu);
	rc = push((void ***)&c->val, &c->nval, &c->capval, r);
	pthread_mutex_unlock(&c->mu);
	return rc;
}

NET2_EXPORT int
net2_sc_collector_tick(struct net2_sc_collector *c, size_t *nhash,
    size_t *nsign, size_t *nvalidate)
{
	struct net2_sc_hash_req **hp;
	struct net2_sc_sign_req **sp, *sreq = NULL;
	struct net2_sc_validate_req **vp, *vreq = NULL;
	size_t nh, ns, nv;
	int rc;

	if (c == NULL)
		return EINVAL;
	/* take the tick's requests; later adds go to the next tick */
	pthread_mutex_lock(&c->mu);
	hp = c->hash;
	nh = c->nhash;
	c->hash = NULL;
	c->nhash = c->caphash = 0;
	sp = c->sign;
	ns = c->nsign;
	vp = c->val;
	nv = c->nval;
	c->sign = NULL;
	c->nsign = c->capsign = 0;
	c->val = NULL;
	c->nval = c->capval = 0;
	pthread_mutex_unlock(&c->mu);
	if (nhash != NULL)
		*nhash = nh;
	if (nsign != NULL)
		*nsign = ns;
	if (nvalidate != NULL)
		*nvalidate = nv;
	/* the tick works on copies, results are written back */
	sreq = malloc((ns + 1) * sizeof(*sreq));
	vreq = malloc((nv + 1) * sizeof(*vreq));
	if (sreq == NULL || vreq == NULL) {
		for (size_t i = 0; i < ns; i++)
			sp[i]->rc = ENOMEM;
		for (size_t i = 0; i < nv; i++)
			vp[i]->result = EIO;
		for (size_t i = 0; i < nh; i++) {
			hp[i]->rc = ENOMEM;
			hp[i]->digestlen = 0;
			if (hp[i]->done != NULL)
				hp[i]->done(hp[i], hp[i]->arg);
		}
		rc = ENOMEM;
		goto out;
	}
	for (size_t i = 0; i < ns; i++)
		sreq[i] = *sp[i];
	for (size_t i = 0; i < nv; i++)
		vreq[i] = *vp[i];
	rc = tick(hp, nh, sreq, ns, vreq, nv, c->nthreads);
	for (size_t i = 0; i < ns; i++)
		sp[i]->rc = sreq[i].rc;
	for (size_t i = 0; i < nv; i++)
		vp[i]->result = vreq[i].result;
out:
	free(sreq);
	free(vreq);
	free(hp);
	free(sp);
	free(vp);
	return rc;
}
