#!/bin/bash
# r06: short-hop kernel times beside the sweep hops (13 pairs, the grid's
# cells moved to the short hops), then the bench line on the r06d PMC profile.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=gpurun_out/short_hop_times.jsonl
: > $out
for args in "--nfft 512" "--nfft 512 --hop-map 128:32,256:64" "--nfft 1024" "--nfft 1024 --hop-map 128:64,256:64"; do
  timeout -k 10 240 python -u tools/time_enhance.py --pairs 13 --reps 5 $args >> $out 2> gpurun_out/short_hop_times.err \
    || { echo "time_enhance $args failed"; tail -5 gpurun_out/short_hop_times.err; exit 1; }
  tail -1 $out
done
timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/bench.json; exit $rc
