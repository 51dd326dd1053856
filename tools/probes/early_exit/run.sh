#!/bin/bash
# GPU box: the isolated early-exit loop, then hex_range over the failing cells of round 4 with the
# round-4 headers (kring_old) and today's (kring_new), each diffed against the host build's output.
cd "$(dirname "$0")"
O=$GRAFT_REPO_ROOT/gpurun_out/early_exit
mkdir -p $O
timeout -k 10 60 ./early_exit > $O/isolated.txt 2>&1 || exit 1
timeout -k 10 60 ./kring_old cells.txt > $O/old_gpu.txt 2>&1 || exit 1
timeout -k 10 60 ./kring_new cells.txt > $O/new_gpu.txt 2>&1 || exit 1
echo "old vs host: $(diff host_out.txt $O/old_gpu.txt | grep -c '^>') rows differ" > $O/summary.txt
echo "new vs host: $(diff host_out.txt $O/new_gpu.txt | grep -c '^>') rows differ" >> $O/summary.txt
cat $O/isolated.txt $O/summary.txt
