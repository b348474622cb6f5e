#!/bin/bash
# FK26 / LV1 training legs, previous library vs this one, interleaved
set -e
O=gpurun_out/r6_zh
mkdir -p $O
for r in 1 2 3 4; do
  KANODE_LIB=$PWD/tools/bin/var/libkanode_base.so timeout -k 10 120 python3 -u tools/legs.py fk26_train lv1_train --reps 40 >> $O/base.jsonl 2>> $O/err.txt
  timeout -k 10 120 python3 -u tools/legs.py fk26_train lv1_train --reps 40 >> $O/new.jsonl 2>> $O/err.txt
done
