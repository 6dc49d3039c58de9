#!/bin/bash
# r06 final profile: kernel traces + PMC passes of the product build (its
# sources changed again, its ISA did not), then the generic kernel's launch
# time on the 13-pair grid moved to 512/160 and 1024/512.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-r06e} bash tools/r06_call3.sh || exit $?
out=gpurun_out/generic_times.jsonl
: > $out
for args in "--nfft 512 --hop-map 128:160,256:160" "--nfft 1024 --hop-map 128:512,256:512"; do
  timeout -k 10 300 python -u tools/time_enhance.py --pairs 13 --reps 3 $args >> $out 2> gpurun_out/generic_times.err \
    || { echo "time_enhance $args failed"; tail -5 gpurun_out/generic_times.err; exit 1; }
  tail -1 $out
done
