#!/bin/bash
# Coalescer measurements on the GPU box (run through gpurun from the repo
# root): the single-message latency / throughput table for 1, 8 and 64
# threads (1 KiB SHA-512 and SHA-256), both staging modes, and a rocprofv3
# trace of single calls (kernel vs copies) for the latency breakdown.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/coalesce
mkdir -p $OUT
B=tools/coalesce_bench
# job forms: 1 = one wave per job (latency form), 2 = one lane per job
for jm in ${JOBMODES:-1 2}; do
	for alg in 3 1; do
		NET2_COALESCE_JOBMODE=$jm timeout -k 10 120 $B $alg 1024 2 1 8 64 \
		    > $OUT/table_jm${jm}_alg${alg}.jsonl || exit $?
		sed "s/^/jobmode=$jm /" $OUT/table_jm${jm}_alg${alg}.jsonl
	done
done
for jm in ${JOBMODES:-1 2}; do
	NET2_COALESCE_JOBMODE=$jm timeout -k 10 120 rocprofv3 --kernel-trace \
	    --memory-copy-trace --stats -d $OUT/trace_jm$jm -o run -- \
	    $B 3 1024 1 1 > $OUT/trace_jm$jm.log 2>&1 || exit $?
done
find $OUT -name "*stats*.csv" | head -20
