#!/bin/bash
# SQ counter passes of the K3 kernels for several library builds (LIBS, each
# a path or "default"), one rocprofv3 run per (build, counter group).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
G1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
G2="SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVES"
for lib in ${LIBS:-default}; do
	tag=$(basename "$lib" .so)
	for g in 1 2; do
		ctrs=$G1; [ $g = 2 ] && ctrs=$G2
		out=gpurun_out/pmc_cmp/$tag/g$g
		mkdir -p "$out"
		if [ "$lib" = default ]; then unset SYZSIG_LIB; else export SYZSIG_LIB=$lib; fi
		timeout -s KILL 240 rocprofv3 --pmc $ctrs --kernel-include-regex "${PMC_KERNELS:-k_agg<|k_agg_scatter}" -f csv \
			-d "$out" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-min > "$out.log" 2>&1
		rc=$?
		echo "[pmc $tag g$g] exit $rc" | tee -a gpurun_out/pmc_cmp/status.log
		[ $rc -ne 0 ] && exit $rc
	done
done
exit 0
