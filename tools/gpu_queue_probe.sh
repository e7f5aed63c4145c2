# stream pairs vs GPU_MAX_HW_QUEUES (tools/queue_pair_probe.py)
for q in 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u tools/queue_pair_probe.py >> gpurun_out/queue_pair2.txt 2>&1 || exit 1
done
cat gpurun_out/queue_pair2.txt
