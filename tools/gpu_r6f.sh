#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/dbg_prefetch5.py 20 A F G I > gpurun_out/dbg5.log 2>&1; grep -v amdgpu.ids gpurun_out/dbg5.log
for r in 1 2; do
  for spec in "-" "contrastive.FUSED=False"; do
    if [ "$spec" = "-" ]; then args=(); else args=($spec); fi
    line=$(timeout -k 10 300 python tools/ab_attr.py "${args[@]}" -- --no-cpu-baseline --steps 40 --workload simclr 2>gpurun_out/abx.err) || { tail -3 gpurun_out/abx.err; exit 1; }
    echo "simclr [$spec] $(echo "$line" | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/ab_xent.txt
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c4 -o run -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 20 --workload simclr > $GRAFT_REPO_ROOT/gpurun_out/prof_c4.json 2>&1; echo "prof rc=$?"
