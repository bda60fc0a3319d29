// common.h -- definitions shared by host and device code of libsyzsig.
//
// Slot encoding of a device-resident Signal (pkg/signal/signal.go:17,
// `type Signal map[elemType]prioType`), one u64 per slot:
//
//      63            32 31      10   9        8       7       0
//     +----------------+----------+--------+---------+---------+
//     |  elem (u32)    |    0     |HASPRIO | PRESENT | prio^0x80|
//     +----------------+----------+--------+---------+---------+
//
// slot == 0 is EMPTY.  A live entry has PRESENT|HASPRIO, so for one key the
// unsigned order of slot words equals the signed order of prio (int8 biased by
// 0x80): atomicMax on the whole word is exactly the max-prio Merge rule of
// signal.go:117-131.  PRESENT without HASPRIO is the batch-transient "absent at
// batch start" marker used by triage (it orders below every live prio, as Go's
// `!ok` does in DiffRaw, signal.go:93).
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define SYZ_HD __host__ __device__ __forceinline__
#else
#define SYZ_HD static inline
#endif

namespace syz {

// 2 x u64 = one 16-B bucket: the common lookup is ONE dwordx4 request per lane
// (scattered-request rate, not bytes, bounds an L2-resident probe).
constexpr uint32_t kBucketShift = 1;
constexpr uint32_t kBucketSlots = 1u << kBucketShift;
constexpr uint64_t kSlotEmpty = 0;
constexpr uint32_t kStatePresent = 0x100;
constexpr uint32_t kStateHasPrio = 0x200;
constexpr uint32_t kStateLive = kStatePresent | kStateHasPrio;

SYZ_HD uint64_t make_slot(uint32_t key, int8_t prio)
{
	return ((uint64_t)key << 32) | kStateLive | (uint32_t)((uint8_t)prio ^ 0x80u);
}
SYZ_HD uint64_t make_absent(uint32_t key) { return ((uint64_t)key << 32) | kStatePresent; }
// Bits 10..28 of a slot word carry a triage-run hint (csrc/triage.hip): zero
// outside a run, cleared by the run's committers.  slot_state() masks it off.
constexpr uint64_t kHintMask = 0x7FFFFull << 10;
SYZ_HD uint32_t slot_state(uint64_t s) { return (uint32_t)s & 0x3FF; }
SYZ_HD uint32_t slot_key(uint64_t s) { return (uint32_t)(s >> 32); }
SYZ_HD bool slot_live(uint64_t s) { return (s & kStateHasPrio) != 0; }
SYZ_HD int8_t slot_prio(uint64_t s) { return (int8_t)((uint8_t)s ^ 0x80u); }
SYZ_HD uint32_t prio_biased(int8_t p) { return (uint8_t)p ^ 0x80u; }

// murmur3 fmix32: bucket index of an element inside one table.
SYZ_HD uint32_t fmix32(uint32_t h)
{
	h ^= h >> 16;
	h *= 0x85ebca6bu;
	h ^= h >> 13;
	h *= 0xc2b2ae35u;
	h ^= h >> 16;
	return h;
}

// fmix32 inverted (a bijection of u32): records that keep bits of h = fmix32(e)
// recover e from them (agg.hip, recs.hip).
SYZ_HD uint32_t fmix32_inv(uint32_t h)
{
	h ^= h >> 16;
	h *= 0x7ed1b41du;  // 0xc2b2ae35^-1 mod 2^32
	h ^= (h >> 13) ^ (h >> 26);
	h *= 0xa5cb9243u;  // 0x85ebca6b^-1 mod 2^32
	h ^= h >> 16;
	return h;
}
static_assert(0x85ebca6bu * 0xa5cb9243u == 1u, "fmix32_inv multiplier");
static_assert(0xc2b2ae35u * 0x7ed1b41du == 1u, "fmix32_inv multiplier");

// Owner shard of an element in an N-way hash-partitioned maxSignal.  Independent
// of fmix32 (different multiplier/offset), so slots stay uniform inside a shard.
SYZ_HD uint32_t owner_of(uint32_t e, uint32_t nshards)
{
	uint32_t h = fmix32(e * 0x9E3779B1u + 0x7F4A7C15u);
	return (uint32_t)(((uint64_t)h * nshards) >> 32);
}

// executor/executor.h:677-685 -- the edge hash of the reference executor.
SYZ_HD uint32_t exec_hash(uint32_t a)
{
	a = (a ^ 61) ^ (a >> 16);
	a = a + (a << 3);
	a = a ^ (a >> 4);
	a = a * 0x27d4eb2du;
	a = a ^ (a >> 15);
	return a;
}

// executor/executor_linux.cc:196-204 (x86_64 text/modules range).
SYZ_HD bool cover_check(uint64_t pc)
{
	return pc >= 0xffffffff80000000ull && pc < 0xffffffffff000000ull;
}

constexpr uint32_t kDedupSize = 8u << 10;   // executor.h:687 dedup_table_size
constexpr uint32_t kCoverSize = 256u << 10; // executor.h:25 kCoverSize (per-call PC limit)

// ---------------------------------------------------------------------------
// Synthetic KCOV workload (DESIGN.md "Workload").  Deterministic and identical
// on host and device, so host checkers and device kernels see the same traces.
// ---------------------------------------------------------------------------

SYZ_HD uint64_t splitmix64(uint64_t* s)
{
	uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
	return z ^ (z >> 31);
}

SYZ_HD uint64_t seed_mix(uint64_t seed, uint64_t a, uint64_t b)
{
	uint64_t s = seed ^ (a * 0xD1B54A32D192ED03ull) ^ (b * 0xAEF17502108EF2D9ull);
	splitmix64(&s);
	return s;
}

constexpr uint64_t kPcBase = 0xffffffff81000000ull;

struct SynthCfg {
	uint64_t seed;          // 20181015 in every config
	uint32_t nblocks_log2;  // basic blocks B = 2^nblocks_log2 (20)
	uint32_t region_log2;   // per-syscall region W = 2^region_log2 blocks (8)
	uint32_t nsys;          // distinct syscalls (4096)
	uint32_t skew;          // 0 uniform syscall choice, 1 power-skewed (u^4), 2 Zipf(1.1) (synth_zipf4096)
	uint32_t restart_log2;  // walk returns to the syscall entry w.p. 2^-restart_log2 (5)
	uint32_t errno_permille;// call fails (errno != 0) w.p. /1000 (300)
	uint32_t any_permille;  // call contains an ANY pointer w.p. /1000 (100)
	uint32_t bad_pc_ppm;    // out-of-range PC rate per PC, parts per million (0)
	uint32_t global_walk;   // 1: SURVEY 8(d)'s walk over all B blocks from a uniform start (0)
};

SYZ_HD uint64_t synth_pc(uint32_t block) { return kPcBase + 5ull * block; }

// Entry block of syscall s.
SYZ_HD uint32_t synth_entry(const SynthCfg& c, uint32_t s)
{
	return fmix32(s * 0x9E3779B1u + 0x01234567u) & ((1u << c.nblocks_log2) - 1);
}

// Zipf(s = 1.1) rank in 1..4096 from 32 random bits (C5's walks
// start from a Zipf(1.1) entry), in integer arithmetic only, so host and
// device draw the same ranks.  Inverse CDF of the power law x^-1.1 on
// [0.5, 4096.5), rounded to the nearest rank: P(k) is proportional to
// (k - 0.5)^-0.1 - (k + 0.5)^-0.1, i.e. 0.1 k^-1.1 to within 1 % for k >= 3
// (rank 1: about 10 % above).  x = t^-10 with t = a - u (a - b), a = 0.5^-0.1,
// b = 4096.5^-0.1, t in Q31 fixed point (t < 2, so every square fits 64 bits).
SYZ_HD uint32_t synth_zipf4096(uint32_t r)
{
	constexpr uint64_t kA = 2301615985ull, kAB = 1366880845ull;  // a and a - b in Q31
	const uint64_t t = kA - ((kAB * r) >> 32);
	const uint64_t t2 = (t * t) >> 31, t4 = (t2 * t2) >> 31, t8 = (t4 * t4) >> 31, t10 = (t8 * t2) >> 31;
	const uint64_t x = ((1ull << 62) / t10 + (1ull << 30)) >> 31;  // round(t^-10)
	return x < 1 ? 1u : x > 4096 ? 4096u : (uint32_t)x;
}

struct SynthCall {
	uint32_t sysno;
	uint8_t failed;  // errno != 0
	uint8_t any;     // prog.CallContainsAny
};

SYZ_HD SynthCall synth_call(const SynthCfg& c, uint64_t prog, uint32_t call)
{
	uint64_t s = seed_mix(c.seed, prog, 0x100000000ull + call);
	uint64_t r = splitmix64(&s);
	SynthCall sc;
	if (c.skew == 2) {
		sc.sysno = (synth_zipf4096((uint32_t)(r >> 32)) - 1) % c.nsys;
	} else if (c.skew) {
		uint64_t x = (r >> 40) & 0xFFFFFF;  // u in [0,1) as 24-bit fixed point
		uint64_t t = (x * x) >> 24;
		t = (t * t) >> 24;                  // u^4
		sc.sysno = (uint32_t)((t * c.nsys) >> 24);
	} else {
		sc.sysno = (uint32_t)(r % c.nsys);
	}
	uint64_t r2 = splitmix64(&s);
	sc.failed = (uint8_t)((r2 % 1000) < c.errno_permille);
	sc.any = (uint8_t)(((r2 >> 20) % 1000) < c.any_permille);
	return sc;
}

// syz-fuzzer/fuzzer.go:513-521 signalPrio.
SYZ_HD uint8_t signal_prio(uint8_t failed, uint8_t any)
{
	uint8_t prio = 0;
	if (!failed)
		prio |= 1 << 1;
	if (!any)
		prio |= 1 << 0;
	return prio;
}

// The raw KCOV trace of one call: a walk inside its syscall's region,
// x <- (4x + 1 + r%4) mod W, restarting at the entry w.p. 2^-restart_log2.
SYZ_HD void synth_trace(const SynthCfg& c, uint64_t prog, uint32_t call, uint64_t* out, uint32_t n)
{
	SynthCall sc = synth_call(c, prog, call);
	uint32_t entry = synth_entry(c, sc.sysno);
	uint32_t bmask = (1u << c.nblocks_log2) - 1, wmask = (1u << c.region_log2) - 1;
	uint32_t rmask = (1u << c.restart_log2) - 1;
	uint64_t s = seed_mix(c.seed, prog, call);
	if (c.global_walk) {  // b <- (4b + 1 + r%4) mod B from a uniform block, no restarts
		uint32_t b = (uint32_t)(splitmix64(&s) >> 20) & bmask;
		if (c.skew == 2)  // (C5) from the entry of a Zipf(1.1)-chosen syscall
			b = entry;
		for (uint32_t i = 0; i < n; i++) {
			uint64_t r = splitmix64(&s);
			uint64_t pc = synth_pc(b);
			if (c.bad_pc_ppm && ((r >> 40) % 1000000) < c.bad_pc_ppm)
				pc = 0x1000ull + i;
			out[i] = pc;
			b = (4 * b + 1 + (uint32_t)((r >> 8) & 3)) & bmask;
		}
		return;
	}
	uint32_t x = 0;
	for (uint32_t i = 0; i < n; i++) {
		uint64_t r = splitmix64(&s);
		uint64_t pc = synth_pc((entry + x) & bmask);
		if (c.bad_pc_ppm && ((r >> 40) % 1000000) < c.bad_pc_ppm)
			pc = 0x1000ull + i;  // outside cover_check's range: aborts the program
		out[i] = pc;
		if ((r & rmask) == 0)
			x = 0;
		else
			x = (4 * x + 1 + (uint32_t)((r >> 8) & 3)) & wmask;
	}
}

// Element i of the synthetic initial maxSignal M0: the first n_known elements
// enumerate the edge signals of syscalls [0, known_sys) (every in-region edge,
// restart edge and entry signal, exactly as write_coverage_signal would derive
// them), the rest are uniform u32; prio uniform in 0..3.
SYZ_HD uint32_t synth_known_per_sys(const SynthCfg& c) { return (1u << c.region_log2) * 5 + 1; }
// known elements of M0 for `known_sys` syscalls (global walk: the whole edge
// universe -- every block's first-PC signal and its 4 out-edges -- once known_sys > 0)
SYZ_HD uint64_t synth_n_known(const SynthCfg& c, uint64_t known_sys)
{
	if (c.global_walk)
		return known_sys ? 5ull << c.nblocks_log2 : 0;
	return known_sys * synth_known_per_sys(c);
}

SYZ_HD void synth_m0_elem(const SynthCfg& c, uint64_t i, uint64_t n_known, uint32_t* elem, int8_t* prio)
{
	uint64_t s = seed_mix(c.seed ^ 0x4D30u, i, 7);
	uint64_t r = splitmix64(&s);
	*prio = (int8_t)(r & 3);
	if (i >= n_known) {
		*elem = (uint32_t)(r >> 32);
		return;
	}
	uint32_t W = 1u << c.region_log2, bmask = (1u << c.nblocks_log2) - 1;
	if (c.global_walk) {
		const uint64_t B = 1ull << c.nblocks_log2;
		if (i < B) {  // a call starting at block i: sig = pc ^ 0
			*elem = (uint32_t)synth_pc((uint32_t)i);
			return;
		}
		const uint32_t x = (uint32_t)((i - B) >> 2), j = (uint32_t)((i - B) & 3);
		*elem = (uint32_t)synth_pc((4 * x + 1 + j) & bmask) ^ exec_hash((uint32_t)synth_pc(x));
		return;
	}
	uint32_t per = synth_known_per_sys(c);
	uint32_t sys = (uint32_t)(i / per), k = (uint32_t)(i % per);
	uint32_t entry = synth_entry(c, sys);
	if (k == 0) {  // first PC of a call: sig = pc ^ 0
		*elem = (uint32_t)synth_pc(entry);
		return;
	}
	k -= 1;
	uint32_t x = k / 5, j = k % 5;
	uint32_t from = (uint32_t)synth_pc((entry + x) & bmask);
	uint32_t to_x = j < 4 ? ((4 * x + 1 + j) & (W - 1)) : 0;  // j == 4: restart edge
	*elem = (uint32_t)synth_pc((entry + to_x) & bmask) ^ exec_hash(from);
}

}  // namespace syz
