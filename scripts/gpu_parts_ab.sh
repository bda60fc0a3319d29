#!/bin/bash
# Partition count x scatter block width on the C2 headline (both trace
# distributions) and the Minimize line: 2048 partitions (64-B blocks), 1024
# partitions with 128-B blocks, 1024 with 64-B blocks (exp build), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/parts
mkdir -p $O
A="--steps 10 --warmup 4 --no-cpu --no-c5 --no-c4 --no-c1 --no-gw --no-pipe"
for rep in 1 2; do
	for v in base p1024 p1024n; do
		case $v in
		base) E="" ;;
		p1024) E="SYZSIG_AGG_PARTS=1024" ;;
		p1024n) E="SYZSIG_AGG_PARTS=1024 SYZSIG_LIB=exp/libsyzsig_narrow.so" ;;
		esac
		for w in global region; do
			X=""; [ $w = region ] && X="--no-min"
			timeout -k 10 300 env $E python -u bench.py $A --walk $w $X > $O/${v}_${w}_$rep.log 2>&1
			rc=$?; echo "[$v $w $rep] exit $rc" >> $O/status.log; [ $rc -ne 0 ] && exit $rc
		done
	done
done
exit 0
