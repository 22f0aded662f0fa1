#!/bin/bash
set -u
O=gpurun_out/${1:-det_probe2}; mkdir -p $O
for v in "nchw bench0 bf16" "nchw bench0 fp16" "cl bench0 fp16"; do
  timeout -k 10 300 python3 tools/det_probe.py $v >> $O/probe.txt 2> $O/probe_$(echo $v | tr ' ' _).err || exit 1
done
cat $O/probe.txt
