#!/bin/bash
# PMC passes (tools/pmc_sets_mem.txt) over a standalone binary.  usage: TAG BINARY [args]
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmc && export TMPDIR=/tmp
TAG=$1; shift
guard() { rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc=$rc"; exit $rc; fi; }
i=0
while read -r CTRS; do
  [ -z "$CTRS" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/pmc/$TAG/p$i -o $TAG -- "$@" > gpurun_out/pmc/$TAG.p$i.log 2>&1; rc=$?; echo "$TAG pass $i rc=$rc"; guard $rc
done < ${SETS:-tools/pmc_sets_mem.txt}
