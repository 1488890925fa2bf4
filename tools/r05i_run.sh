#!/bin/bash
# round 5 final evidence (one build): GPU suite, heavy + whole-product PMC (copied into profiles/ first, so the bench
# line's traffic fields come from this build), the N = 1 bench line as the driver runs it, rocprofv3 kernel stats, SQ
set -u
T=r05i
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
tools/gpu_steps.sh $T tests pmc || exit $?
cp $OUT/${T}_pmc_heavy.json profiles/${T}_pmc_heavy.json && cp $OUT/${T}_pmc_product.json profiles/${T}_pmc_product.json || exit 20
tools/gpu_steps.sh $T bench:--steps,20,--warmup,5 prof sq || exit $?
