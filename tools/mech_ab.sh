#!/bin/bash
# Round-5 verdict item 3: each perf mechanism against its removal, alternated
# on one box in the driver's regimes (tools/variants_ab.py): the headline
# (bench.py 20/5, fresh process per run) and cycles 1 s apart (the daemon).
#   base   - the default (workers follow the cycle thread's L3 domain; loop
#            writes rewrite the swapped-out file)
#   none   - --cpu-affinity=none (no placement at all)
#   l3     - --cpu-affinity=l3 (daemon only: the whole process on one L3)
#   plain  - every loop write creates a new temporary file and renames it
#            over the feature file (the reference's write), through an
#            experiment switch (GFD_EXP_WRITER) of the tree the A/B ran on,
#            removed before it was committed: on later trees this variant
#            runs the default writer.  Its numbers: profiles/mechanisms_ab_r5.txt.
set -o pipefail
out=gpurun_out/${1:-mech_ab}
mkdir -p "$out"
timeout -k 10 400 python3 -u tools/variants_ab.py --modes headline --reps 5 \
  --variant base= --variant none=GFD_CPU_AFFINITY=none --variant plain=GFD_EXP_WRITER=plain > "$out/headline.jsonl" &&
timeout -k 10 600 python3 -u tools/variants_ab.py --modes cold --reps 4 --cold-cycles 10 \
  --variant base= --variant none=GFD_CPU_AFFINITY=none --variant l3=GFD_CPU_AFFINITY=l3 \
  --variant plain=GFD_EXP_WRITER=plain > "$out/cold.jsonl" &&
grep summary "$out/headline.jsonl" "$out/cold.jsonl" | cut -c1-220
