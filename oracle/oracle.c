/*
 * oracle.c -- CPU restatement of the reference's coverage-signal hot path.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Plain C, single-threaded,
 * written for clarity and literal fidelity, not speed.
 */
#include "oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ======================= executor half ======================= */

/* executor/executor.h:677-685 */
uint32_t orc_exec_hash(uint32_t a)
{
	a = (a ^ 61) ^ (a >> 16);
	a = a + (a << 3);
	a = a ^ (a >> 4);
	a = a * 0x27d4eb2d;
	a = a ^ (a >> 15);
	return a;
}

/* executor/executor_linux.cc:196-204, the x86_64 branch */
int orc_cover_check(uint64_t pc)
{
	return pc >= 0xffffffff80000000ull && pc < 0xffffffffff000000ull;
}

#define ORC_DEDUP_SIZE (8u << 10) /* executor.h:687 dedup_table_size */

/* executor/executor.h:692-706; table is per program (zeroed by the per-program fork) */
static int orc_dedup(uint32_t* table, uint32_t sig)
{
	for (uint32_t i = 0; i < 4; i++) {
		uint32_t pos = (sig + i) % ORC_DEDUP_SIZE;
		if (table[pos] == sig)
			return 1;
		if (table[pos] == 0) {
			table[pos] = sig;
			return 0;
		}
	}
	table[sig % ORC_DEDUP_SIZE] = sig;
	return 0;
}

/* executor/executor.h:492-512 write_coverage_signal<uint64>, driven per call in
 * completion order (non-threaded: call order) by handle_completion (:530-608). */
void orc_exec_program(const uint64_t* pcs, const uint64_t* call_start, const uint32_t* call_len,
                      uint32_t ncalls, uint32_t* out_sig, uint32_t* out_cnt, uint32_t* completed)
{
	uint32_t* table = (uint32_t*)calloc(ORC_DEDUP_SIZE, sizeof(uint32_t));
	uint32_t done = 0;
	for (uint32_t c = 0; c < ncalls; c++)
		out_cnt[c] = 0;
	for (uint32_t c = 0; c < ncalls; c++) {
		const uint64_t* cover = pcs + call_start[c];
		uint32_t* out = out_sig + call_start[c];
		uint32_t nsig = 0;
		uint64_t prev = 0;
		int aborted = 0;
		for (uint32_t i = 0; i < call_len[c]; i++) {
			uint64_t pc = cover[i];
			if (!orc_cover_check(pc)) { /* doexit(0): this call and the rest publish nothing */
				aborted = 1;
				break;
			}
			uint64_t sig = pc ^ prev;
			prev = orc_exec_hash((uint32_t)pc);
			if (orc_dedup(table, (uint32_t)sig))
				continue;
			out[nsig++] = (uint32_t)sig; /* write_output truncates to uint32 */
		}
		if (aborted)
			break;
		out_cnt[c] = nsig;
		done = c + 1; /* write_completed(completed), executor.h:604 */
	}
	*completed = done;
	free(table);
}

/* ======================= pkg/signal half ======================= */
/* Go map[uint32]int8 restated as an open-addressing table.  Iteration order is
 * slot order (Go's is random; no function below depends on it except Serialize,
 * whose callers compare as sets). */

struct orc_sig {
	uint64_t cap; /* power of two */
	uint64_t len;
	uint32_t* keys;
	int8_t* vals;
	uint8_t* used;
};

static uint32_t orc_mix(uint32_t h)
{
	h ^= h >> 16;
	h *= 0x85ebca6bu;
	h ^= h >> 13;
	h *= 0xc2b2ae35u;
	h ^= h >> 16;
	return h;
}

orc_sig* orc_sig_new(uint64_t hint)
{
	orc_sig* s = (orc_sig*)calloc(1, sizeof(orc_sig));
	uint64_t cap = 16;
	while (cap < 2 * hint)
		cap <<= 1;
	s->cap = cap;
	s->keys = (uint32_t*)calloc(cap, sizeof(uint32_t));
	s->vals = (int8_t*)calloc(cap, sizeof(int8_t));
	s->used = (uint8_t*)calloc(cap, 1);
	return s;
}

void orc_sig_free(orc_sig* s)
{
	if (!s)
		return;
	free(s->keys);
	free(s->vals);
	free(s->used);
	free(s);
}

uint64_t orc_sig_len(const orc_sig* s)
{
	return s ? s->len : 0; /* len(nil map) == 0 */
}

static uint64_t orc_find(const orc_sig* s, uint32_t e)
{
	uint64_t m = s->cap - 1, i = orc_mix(e) & m;
	while (s->used[i] && s->keys[i] != e)
		i = (i + 1) & m;
	return i;
}

int orc_sig_get(const orc_sig* s, uint32_t e, int8_t* p)
{
	if (!s || s->len == 0)
		return 0;
	uint64_t i = orc_find(s, e);
	if (!s->used[i])
		return 0;
	if (p)
		*p = s->vals[i];
	return 1;
}

static void orc_grow(orc_sig* s)
{
	orc_sig n = {0};
	n.cap = s->cap * 2;
	n.keys = (uint32_t*)calloc(n.cap, sizeof(uint32_t));
	n.vals = (int8_t*)calloc(n.cap, sizeof(int8_t));
	n.used = (uint8_t*)calloc(n.cap, 1);
	for (uint64_t i = 0; i < s->cap; i++) {
		if (!s->used[i])
			continue;
		uint64_t j = orc_find(&n, s->keys[i]);
		n.used[j] = 1;
		n.keys[j] = s->keys[i];
		n.vals[j] = s->vals[i];
	}
	n.len = s->len;
	free(s->keys);
	free(s->vals);
	free(s->used);
	*s = n;
}

/* s[e] = p (assignment) */
static void orc_set(orc_sig* s, uint32_t e, int8_t p)
{
	if (2 * (s->len + 1) > s->cap)
		orc_grow(s);
	uint64_t i = orc_find(s, e);
	if (!s->used[i]) {
		s->used[i] = 1;
		s->keys[i] = e;
		s->len++;
	}
	s->vals[i] = p;
}

/* signal.go:31-40 */
orc_sig* orc_from_raw(const uint32_t* raw, uint64_t n, uint8_t prio)
{
	if (n == 0)
		return NULL;
	orc_sig* s = orc_sig_new(n);
	for (uint64_t i = 0; i < n; i++)
		orc_set(s, raw[i], (int8_t)prio);
	return s;
}

/* signal.go:42-57 (empty -> Serial{}; order: slot order) */
uint64_t orc_serialize(const orc_sig* s, uint32_t* elems, int8_t* prios)
{
	uint64_t n = 0;
	if (!s)
		return 0;
	for (uint64_t i = 0; i < s->cap; i++) {
		if (!s->used[i])
			continue;
		elems[n] = s->keys[i];
		prios[n] = s->vals[i];
		n++;
	}
	return n;
}

/* signal.go:59-71: panic("corrupted Serial") on mismatch; later duplicates overwrite */
int orc_deserialize(const uint32_t* elems, uint64_t ne, const int8_t* prios, uint64_t np,
                    orc_sig** out)
{
	*out = NULL;
	if (ne != np)
		return -1;
	if (ne == 0)
		return 0;
	orc_sig* s = orc_sig_new(ne);
	for (uint64_t i = 0; i < ne; i++)
		orc_set(s, elems[i], prios[i]);
	*out = s;
	return 0;
}

/* signal.go:73-88 */
orc_sig* orc_diff(const orc_sig* s, const orc_sig* s1)
{
	if (orc_sig_len(s1) == 0)
		return NULL;
	orc_sig* res = NULL;
	for (uint64_t i = 0; i < s1->cap; i++) {
		if (!s1->used[i])
			continue;
		uint32_t e = s1->keys[i];
		int8_t p1 = s1->vals[i], p;
		if (orc_sig_get(s, e, &p) && p >= p1)
			continue;
		if (!res)
			res = orc_sig_new(0);
		orc_set(res, e, p1);
	}
	return res;
}

/* signal.go:90-102 (prio compared as int8) */
orc_sig* orc_diff_raw(const orc_sig* s, const uint32_t* raw, uint64_t n, uint8_t prio)
{
	orc_sig* res = NULL;
	int8_t pr = (int8_t)prio, p;
	for (uint64_t i = 0; i < n; i++) {
		if (orc_sig_get(s, raw[i], &p) && p >= pr)
			continue;
		if (!res)
			res = orc_sig_new(0);
		orc_set(res, raw[i], pr);
	}
	return res;
}

/* signal.go:104-115: nil if s1 empty, else non-nil (possibly empty) */
orc_sig* orc_intersection(const orc_sig* s, const orc_sig* s1)
{
	if (orc_sig_len(s1) == 0)
		return NULL;
	orc_sig* res = orc_sig_new(orc_sig_len(s));
	if (!s)
		return res;
	for (uint64_t i = 0; i < s->cap; i++) {
		if (!s->used[i])
			continue;
		int8_t p1;
		if (orc_sig_get(s1, s->keys[i], &p1) && p1 >= s->vals[i])
			orc_set(res, s->keys[i], s->vals[i]);
	}
	return res;
}

/* signal.go:117-131: max-prio merge; allocates a nil receiver */
void orc_merge(orc_sig** sp, const orc_sig* s1)
{
	if (orc_sig_len(s1) == 0)
		return;
	if (!*sp)
		*sp = orc_sig_new(s1->len);
	orc_sig* s = *sp;
	for (uint64_t i = 0; i < s1->cap; i++) {
		if (!s1->used[i])
			continue;
		int8_t p;
		if (!orc_sig_get(s, s1->keys[i], &p) || p < s1->vals[i])
			orc_set(s, s1->keys[i], s1->vals[i]);
	}
}

/* ---- signal.go:138-166 Minimize ---- */

static const uint64_t* g_sort_len;
static int orc_cmp_ctx(const void* a, const void* b)
{
	uint64_t i = *(const uint64_t*)a, j = *(const uint64_t*)b;
	if (g_sort_len[i] != g_sort_len[j])
		return g_sort_len[i] > g_sort_len[j] ? -1 : 1; /* Len() desc, signal.go:139-141 */
	return i < j ? -1 : (i > j); /* fixed tie order (reference: unstable sort.Slice) */
}

/* covered map[elemType]ContextPrio (signal.go:142-146) */
typedef struct {
	uint64_t cap, len;
	uint32_t* keys;
	int8_t* prio;
	uint64_t* idx;
	uint8_t* used;
} orc_cov;

static uint64_t orc_cov_find(const orc_cov* m, uint32_t e)
{
	uint64_t mask = m->cap - 1, i = orc_mix(e) & mask;
	while (m->used[i] && m->keys[i] != e)
		i = (i + 1) & mask;
	return i;
}

static void orc_cov_init(orc_cov* m, uint64_t cap)
{
	m->cap = cap;
	m->len = 0;
	m->keys = (uint32_t*)calloc(cap, sizeof(uint32_t));
	m->prio = (int8_t*)calloc(cap, 1);
	m->idx = (uint64_t*)calloc(cap, sizeof(uint64_t));
	m->used = (uint8_t*)calloc(cap, 1);
}

static void orc_cov_release(orc_cov* m)
{
	free(m->keys);
	free(m->prio);
	free(m->idx);
	free(m->used);
}

static void orc_cov_grow(orc_cov* m)
{
	orc_cov n;
	orc_cov_init(&n, m->cap * 2);
	for (uint64_t i = 0; i < m->cap; i++) {
		if (!m->used[i])
			continue;
		uint64_t j = orc_cov_find(&n, m->keys[i]);
		n.used[j] = 1;
		n.keys[j] = m->keys[i];
		n.prio[j] = m->prio[i];
		n.idx[j] = m->idx[i];
	}
	n.len = m->len;
	orc_cov_release(m);
	*m = n;
}

uint64_t orc_minimize(const uint64_t* ctx_off, const uint32_t* elems, const int8_t* prios,
                      uint64_t nctx, uint64_t* out_idx)
{
	uint64_t* order = (uint64_t*)malloc((nctx + 1) * sizeof(uint64_t));
	uint64_t* lens = (uint64_t*)malloc((nctx + 1) * sizeof(uint64_t));
	for (uint64_t i = 0; i < nctx; i++) {
		order[i] = i;
		lens[i] = ctx_off[i + 1] - ctx_off[i];
	}
	g_sort_len = lens;
	qsort(order, nctx, sizeof(uint64_t), orc_cmp_ctx);
	orc_cov cov;
	orc_cov_init(&cov, 1024);
	for (uint64_t si = 0; si < nctx; si++) { /* for i, inp := range corpus (sorted) */
		uint64_t c = order[si];
		for (uint64_t j = ctx_off[c]; j < ctx_off[c + 1]; j++) {
			if (2 * (cov.len + 1) > cov.cap)
				orc_cov_grow(&cov);
			uint64_t s = orc_cov_find(&cov, elems[j]);
			if (!cov.used[s]) { /* !ok */
				cov.used[s] = 1;
				cov.keys[s] = elems[j];
				cov.len++;
			} else if (!(prios[j] > cov.prio[s])) { /* p > prev.prio */
				continue;
			}
			cov.prio[s] = prios[j];
			cov.idx[s] = si;
		}
	}
	/* indices := set of covered[e].idx (signal.go:157-160); result = their Contexts */
	uint8_t* win = (uint8_t*)calloc(nctx + 1, 1);
	for (uint64_t s = 0; s < cov.cap; s++)
		if (cov.used[s])
			win[order[cov.idx[s]]] = 1;
	orc_cov_release(&cov);
	uint64_t n = 0;
	for (uint64_t i = 0; i < nctx; i++)
		if (win[i])
			out_idx[n++] = i;
	free(win);
	free(order);
	free(lens);
	return n;
}

/* ---- syz-fuzzer/fuzzer.go:494-511 checkNewSignal, over a batch in serial order ---- */
void orc_triage_batch(orc_sig** max_signal, orc_sig** new_signal, const uint32_t* sigs,
                      const uint64_t* call_start, const uint32_t* call_len, const uint8_t* call_prio,
                      uint64_t ncalls, uint32_t* new_bits, uint8_t* call_new)
{
	for (uint64_t k = 0; k < ncalls; k++) {
		const uint32_t* raw = sigs + call_start[k];
		call_new[k] = 0;
		orc_sig* diff = orc_diff_raw(*max_signal, raw, call_len[k], call_prio[k]);
		if (orc_sig_len(diff) == 0) {
			orc_sig_free(diff);
			continue;
		}
		call_new[k] = 1;
		for (uint32_t i = 0; i < call_len[k]; i++) {
			if (orc_sig_get(diff, raw[i], NULL)) {
				uint64_t r = call_start[k] + i;
				new_bits[r >> 5] |= 1u << (r & 31);
			}
		}
		orc_merge(max_signal, diff);
		orc_merge(new_signal, diff);
		orc_sig_free(diff);
	}
}

/* ---- multi-core CPU baseline: fuzzer.go:494-511 as `procs` goroutines run it ----
 * nthreads workers (the fuzzer's Procs, fuzzer.go:288-295) take programs in
 * order; per call: DiffRaw under signalMu.RLock, and when non-empty the
 * RUnlock/Lock upgrade, maxSignal.Merge + newSignal.Merge, Unlock/RLock
 * (fuzzer.go:494-511).  Like the reference, the interleaving of the procs
 * makes which call reports a shared new element nondeterministic; the final
 * maxSignal is deterministic (max is order-independent).  Timing baseline only. */
typedef struct {
	orc_sig** ms;
	orc_sig** ns;
	const uint32_t* sigs;
	const uint64_t* call_start;
	const uint32_t* call_len;
	const uint8_t* call_prio;
	uint64_t nprog, calls_per_prog;
	uint64_t next; /* next program (atomic) */
	uint64_t ncalls_new;
	pthread_rwlock_t mu; /* fuzzer.signalMu */
} orc_mt;

static void* orc_mt_proc(void* arg)
{
	orc_mt* m = (orc_mt*)arg;
	uint64_t nnew = 0;
	for (;;) {
		uint64_t p = __atomic_fetch_add(&m->next, 1, __ATOMIC_RELAXED);
		if (p >= m->nprog)
			break;
		pthread_rwlock_rdlock(&m->mu);
		for (uint64_t k = p * m->calls_per_prog; k < (p + 1) * m->calls_per_prog; k++) {
			orc_sig* diff = orc_diff_raw(*m->ms, m->sigs + m->call_start[k], m->call_len[k], m->call_prio[k]);
			if (orc_sig_len(diff) == 0) {
				orc_sig_free(diff);
				continue;
			}
			nnew++;
			pthread_rwlock_unlock(&m->mu);
			pthread_rwlock_wrlock(&m->mu);
			orc_merge(m->ms, diff);
			orc_merge(m->ns, diff);
			pthread_rwlock_unlock(&m->mu);
			pthread_rwlock_rdlock(&m->mu);
			orc_sig_free(diff);
		}
		pthread_rwlock_unlock(&m->mu);
	}
	__atomic_fetch_add(&m->ncalls_new, nnew, __ATOMIC_RELAXED);
	return NULL;
}

uint64_t orc_triage_batch_mt(orc_sig** max_signal, orc_sig** new_signal, const uint32_t* sigs,
                             const uint64_t* call_start, const uint32_t* call_len, const uint8_t* call_prio,
                             uint64_t nprog, uint64_t calls_per_prog, uint32_t nthreads)
{
	orc_mt m;
	memset(&m, 0, sizeof(m));
	m.ms = max_signal;
	m.ns = new_signal;
	m.sigs = sigs;
	m.call_start = call_start;
	m.call_len = call_len;
	m.call_prio = call_prio;
	m.nprog = nprog;
	m.calls_per_prog = calls_per_prog;
	pthread_rwlock_init(&m.mu, NULL);
	if (!*max_signal) /* the zero-value maxSignal is usable: Merge allocates (signal.go:121-125) */
		*max_signal = orc_sig_new(0);
	if (nthreads < 1)
		nthreads = 1;
	pthread_t* th = (pthread_t*)calloc(nthreads, sizeof(pthread_t));
	for (uint32_t i = 0; i < nthreads; i++)
		pthread_create(&th[i], NULL, orc_mt_proc, &m);
	for (uint32_t i = 0; i < nthreads; i++)
		pthread_join(th[i], NULL);
	free(th);
	pthread_rwlock_destroy(&m.mu);
	return m.ncalls_new;
}

/* Test helper (not a reference function): the entries of a Serial whose
 * element is in keys[], in input order -- Deserialize of the result agrees
 * with Deserialize of the whole Serial on every key (later duplicates still
 * overwrite earlier ones, signal.go:66-69).  Returns the count written. */
uint64_t orc_filter_keys(const uint32_t* elems, const int8_t* prios, uint64_t n, const uint32_t* keys,
                         uint64_t nkeys, uint32_t* out_e, int8_t* out_p)
{
	orc_sig* set = orc_from_raw(keys, nkeys, 0);
	uint64_t k = 0;
	if (set) {
		for (uint64_t i = 0; i < n; i++) {
			if (orc_sig_get(set, elems[i], NULL)) {
				out_e[k] = elems[i];
				out_p[k] = prios[i];
				k++;
			}
		}
	}
	orc_sig_free(set);
	return k;
}
