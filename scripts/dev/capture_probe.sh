# every (capture mode, other-thread call) of scripts/dev/capture_probe.py in its own process
mkdir -p gpurun_out
: > gpurun_out/capture_probe.jsonl
for mode in thread_local global; do
  for i in 0 1 2 3 4 5 6 7; do
    timeout -k 5 40 python scripts/dev/capture_probe.py $mode $i 2>/dev/null | grep '^{' >> gpurun_out/capture_probe.jsonl
    rc=${PIPESTATUS[0]}
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "{\"mode\": \"$mode\", \"call_index\": $i, \"exit\": $rc}" >> gpurun_out/capture_probe.jsonl; fi
    if [ $rc -ge 124 ]; then exit $rc; fi
  done
done
