// san_driver.cc -- runs the CPU restatement (oracle.c) under the sanitizers
// SURVEY.md section 5 plans for it: AddressSanitizer + UndefinedBehaviorSanitizer
// (`make -C oracle san` -> _san/driver_asan) and ThreadSanitizer for the
// multi-threaded baseline (_san/driver_tsan).  TEST INFRASTRUCTURE ONLY, run by
// tests/test_sanitizers.py.
//
// One synthetic batch (csrc/common.h's KCOV walk, skewed syscalls so the
// rwlock sees contention) goes through every oracle entry point: the executor
// (orc_exec_program per program), checkNewSignal sequentially and as N Procs
// under the rwlock (orc_triage_batch_mt, fuzzer.go:494-511), the Signal ops,
// Serialize/Deserialize and Minimize.  Exit status 0 iff the two triage forms
// end in the same maxSignal and newSignal and every op's invariant holds; the
// sanitizers abort the process on the first error they find.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../syzkaller_amd/csrc/common.h"
#include "oracle.h"

using namespace syz;

static int fails = 0;
#define CHECK(c)                                                  \
	do {                                                          \
		if (!(c)) {                                               \
			fprintf(stderr, "CHECK failed: %s (line %d)\n", #c, __LINE__); \
			fails++;                                              \
		}                                                         \
	} while (0)

static bool same_sig(const orc_sig* a, const orc_sig* b)
{
	if (orc_sig_len(a) != orc_sig_len(b))
		return false;
	const uint64_t n = orc_sig_len(a);
	std::vector<uint32_t> e(n + 1);
	std::vector<int8_t> p(n + 1);
	orc_serialize(a, e.data(), p.data());
	for (uint64_t i = 0; i < n; i++) {
		int8_t q;
		if (!orc_sig_get(b, e[i], &q) || q != p[i])
			return false;
	}
	return true;
}

int main(int argc, char** argv)
{
	const uint32_t nprog = argc > 1 ? (uint32_t)atoi(argv[1]) : 48, cpp = 16, len = 700;
	const uint32_t nthreads = argc > 2 ? (uint32_t)atoi(argv[2]) : 8;
	SynthCfg cfg = {20181015, 20, 8, 4096, 1, 5, 300, 100, 0};
	const uint64_t ncalls = (uint64_t)nprog * cpp;
	std::vector<uint64_t> pcs(ncalls * len), cs(ncalls);
	std::vector<uint32_t> cl(ncalls, len), sigs(ncalls * len), cnt(ncalls);
	std::vector<uint8_t> prio(ncalls);
	for (uint64_t c = 0; c < ncalls; c++) {
		cs[c] = c * len;
		const uint32_t p = (uint32_t)(c / cpp), k = (uint32_t)(c % cpp);
		synth_trace(cfg, p, k, &pcs[cs[c]], len);
		const SynthCall sc = synth_call(cfg, p, k);
		prio[c] = signal_prio(sc.failed, sc.any);
	}
	// executor half, one forked child per program
	for (uint32_t p = 0; p < nprog; p++) {
		uint32_t done = 0;
		std::vector<uint64_t> lcs(cpp);
		for (uint32_t k = 0; k < cpp; k++)
			lcs[k] = (uint64_t)k * len;
		orc_exec_program(&pcs[(uint64_t)p * cpp * len], lcs.data(), &cl[(uint64_t)p * cpp], cpp,
		                 &sigs[(uint64_t)p * cpp * len], &cnt[(uint64_t)p * cpp], &done);
		CHECK(done == cpp);
	}
	// M0
	const uint64_t nm0 = 20000;
	std::vector<uint32_t> m0e(nm0);
	std::vector<int8_t> m0p(nm0);
	for (uint64_t i = 0; i < nm0; i++)
		synth_m0_elem(cfg, i, 64 * synth_known_per_sys(cfg), &m0e[i], &m0p[i]);
	// checkNewSignal: sequential vs Procs under the rwlock
	orc_sig *ms1 = nullptr, *ns1 = nullptr, *ms2 = nullptr, *ns2 = nullptr;
	CHECK(orc_deserialize(m0e.data(), nm0, m0p.data(), nm0, &ms1) == 0);
	CHECK(orc_deserialize(m0e.data(), nm0, m0p.data(), nm0, &ms2) == 0);
	std::vector<uint32_t> bits((sigs.size() + 31) / 32);
	std::vector<uint8_t> cnew(ncalls);
	orc_triage_batch(&ms1, &ns1, sigs.data(), cs.data(), cnt.data(), prio.data(), ncalls, bits.data(), cnew.data());
	const uint64_t nmt = orc_triage_batch_mt(&ms2, &ns2, sigs.data(), cs.data(), cnt.data(), prio.data(), nprog, cpp,
	                                         nthreads);
	CHECK(same_sig(ms1, ms2));
	CHECK(same_sig(ns1, ns2));
	CHECK(nmt > 0 && nmt <= ncalls);
	// Signal ops: Diff / DiffRaw / Intersection / Merge / Serialize round trip
	orc_sig* raw = orc_from_raw(sigs.data(), cnt[0], prio[0]);
	orc_sig* d = orc_diff(ms1, raw);
	CHECK(orc_sig_len(d) == 0);  // everything in the batch is in the final maxSignal
	orc_sig* dr = orc_diff_raw(ms1, sigs.data(), cnt[0], 0x7f);
	orc_sig* in = orc_intersection(ms1, raw);
	CHECK(orc_sig_len(in) == orc_sig_len(raw));
	orc_sig* mg = nullptr;
	orc_merge(&mg, raw);
	orc_merge(&mg, dr);
	CHECK(orc_sig_len(mg) >= orc_sig_len(raw));
	const uint64_t n1 = orc_sig_len(ms1);
	std::vector<uint32_t> se(n1 + 1);
	std::vector<int8_t> sp(n1 + 1);
	CHECK(orc_serialize(ms1, se.data(), sp.data()) == n1);
	orc_sig* back = nullptr;
	CHECK(orc_deserialize(se.data(), n1, sp.data(), n1, &back) == 0);
	CHECK(same_sig(ms1, back));
	// Minimize over the calls' signals as contexts
	std::vector<uint64_t> off(ncalls + 1);
	std::vector<uint32_t> me;
	std::vector<int8_t> mp;
	for (uint64_t c = 0; c < ncalls; c++) {
		off[c] = me.size();
		for (uint32_t i = 0; i < cnt[c]; i++) {
			me.push_back(sigs[cs[c] + i]);
			mp.push_back((int8_t)prio[c]);
		}
	}
	off[ncalls] = me.size();
	std::vector<uint64_t> keep(ncalls);
	const uint64_t nk = orc_minimize(off.data(), me.data(), mp.data(), ncalls, keep.data());
	CHECK(nk > 0 && nk <= ncalls);
	for (uint64_t i = 1; i < nk; i++)
		CHECK(keep[i - 1] < keep[i]);
	for (orc_sig* s : {ms1, ns1, ms2, ns2, raw, d, dr, in, mg, back})
		orc_sig_free(s);
	printf("san_driver: %u programs, %llu calls, %llu records, maxSignal %llu, %llu calls new (%u threads), "
	       "%llu kept by Minimize, %d failures\n",
	       nprog, (unsigned long long)ncalls, (unsigned long long)me.size(), (unsigned long long)n1,
	       (unsigned long long)nmt, nthreads, (unsigned long long)nk, fails);
	return fails ? 1 : 0;
}
