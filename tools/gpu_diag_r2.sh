export TMPDIR=/tmp
mkdir -p gpurun_out
port=29561
for v in "AVDINO_GRAD_BUCKETS=1 X=1" "AVDINO_GRAD_BUCKETS=0 X=1"; do
  env $(echo $v | cut -d' ' -f1) true
  extra=$(echo $v | cut -d' ' -f2 | sed 's/X=1//;s/X=//')
  export $(echo $v | cut -d' ' -f1)
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port $port bench.py --gpus 2 --steps 5 --warmup 3 --batch 128 --mode mse $extra --dist-backend gloo \
      --no-cpu-baseline > gpurun_out/diag.json 2> gpurun_out/diag.err
  rc=$?; echo "$v rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/diag.json) $(grep -o '"host_issue_ms_per_step": [0-9.]*' gpurun_out/diag.json)"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/diag.err; exit $rc; }
  port=$((port+1))
done
