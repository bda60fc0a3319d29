// ref_harness.cc -- drives the REFERENCE executor's own signal code on synthetic
// KCOV traces to produce golden vectors.  TEST INFRASTRUCTURE ONLY.
//
// Built by oracle/Makefile (container only, needs /root/reference) into
// oracle/_ref/ref_harness.  It #includes the reference translation unit
// executor/executor_linux.cc unchanged (its main renamed), so every function that
// runs here -- handle_completion (executor.h:530-608), write_coverage_signal<uint64>
// (:492-528), hash/dedup (:677-706), cover_check/write_output/write_completed
// (executor_linux.cc:196-219) -- is the reference's own code, compiled with the
// reference Makefile's flags (Makefile:139-143).  No reference source is copied.
//
// Protocol (little-endian, stdin):
//   u32 nprog; per program: u32 ncalls; per call: u32 failed (errno != 0), u32 npc, u64 pc[npc]
// Output (stdout): per program: u32 nwords, then the executor's output region
//   words [0, nwords): word 0 = completed count (write_completed), then per
//   completed call the record: callIndex, callNum, errno, faultInjected, nsig,
//   ncover, ncomps, sig[nsig]   (executor.h:566-604).
// Each program runs in a forked child, exactly like the executor's per-program
// fork (common_linux.h:1995-2030): the dedup table starts zeroed, and a
// cover_check failure's doexit(0) ends only that child.
#define main syz_reference_executor_main
#include "executor_linux.cc"
#undef main

#include <sys/mman.h>
#include <vector>

static bool read_exact(void* p, size_t n)
{
	char* c = (char*)p;
	while (n) {
		ssize_t r = read(0, c, n);
		if (r <= 0)
			return false;
		c += r;
		n -= r;
	}
	return true;
}

static void write_exact(const void* p, size_t n)
{
	const char* c = (const char*)p;
	while (n) {
		ssize_t r = write(1, c, n);
		if (r <= 0)
			doexit(2);
		c += r;
		n -= r;
	}
}

struct call_in {
	uint32 failed;
	std::vector<uint64> pcs;
};

int main()
{
	uint32 nprog = 0;
	if (!read_exact(&nprog, 4))
		return 1;
	// Shared output region (kMaxOutput, executor.h:24), like the executor's shmem out file.
	uint32* shared = (uint32*)mmap(0, kMaxOutput, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
	// Per-thread KCOV-like buffer: word 0 = count, words 1.. = PCs (executor_linux.cc:143-149).
	uint64* cover = (uint64*)mmap(0, (kCoverSize + 1) * sizeof(uint64), PROT_READ | PROT_WRITE,
				      MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
	if (shared == MAP_FAILED || cover == MAP_FAILED)
		return 1;
	for (uint32 p = 0; p < nprog; p++) {
		uint32 ncalls = 0;
		if (!read_exact(&ncalls, 4))
			return 1;
		std::vector<call_in> calls(ncalls);
		for (uint32 c = 0; c < ncalls; c++) {
			uint32 hdr[2];
			if (!read_exact(hdr, 8))
				return 1;
			calls[c].failed = hdr[0];
			calls[c].pcs.resize(hdr[1]);
			if (hdr[1] && !read_exact(calls[c].pcs.data(), 8ull * hdr[1]))
				return 1;
		}
		memset(shared, 0, 4096);
		pid_t pid = fork();
		if (pid < 0)
			return 1;
		if (pid == 0) {
			// Child == one executor worker executing one program.
			is_kernel_64_bit = true;
			flag_cover = true;
			flag_collect_cover = false;
			flag_collect_comps = false;
			collide = false;
			output_data = shared;
			output_pos = output_data; // common_linux.h:2026
			write_output(0); // executor.h:297, number of executed syscalls
			thread_t* th = &threads[0];
			th->cover_data = (char*)cover;
			th->cover_end = (char*)(cover + kCoverSize + 1);
			for (uint32 c = 0; c < ncalls; c++) {
				event_init(&th->ready);
				event_init(&th->done);
				event_set(&th->done);
				th->handled = false;
				th->colliding = false;
				th->call_index = c;
				th->call_num = c;
				th->copyout_index = no_copyout;
				th->res = calls[c].failed ? -1 : 0;
				th->reserrno = calls[c].failed ? EINVAL : 0;
				th->fault_injected = false;
				// A successful call reads copyout instructions; give it instr_eof.
				*(uint64*)input_data = instr_eof;
				th->copyout_pos = (uint64*)input_data;
				cover[0] = calls[c].pcs.size();
				memcpy(cover + 1, calls[c].pcs.data(), 8 * calls[c].pcs.size());
				th->cover_size = read_cover_size(th); // executor_linux.cc:179-189
				running = 1;
				handle_completion(th);
			}
			doexit(0);
		}
		int status = 0;
		waitpid(pid, &status, 0);
		if (!WIFEXITED(status) || WEXITSTATUS(status) != 0)
			return 3;
		// Walk the records to find the used length.
		uint32 completed = shared[0];
		uint32 pos = 1;
		for (uint32 r = 0; r < completed; r++) {
			uint32 nsig = shared[pos + 4], ncover = shared[pos + 5], ncomps = shared[pos + 6];
			(void)ncomps; // comps are off (flag_collect_comps = false)
			pos += 7 + nsig + ncover;
		}
		write_exact(&pos, 4);
		write_exact(shared, 4ull * pos);
	}
	return 0;
}
