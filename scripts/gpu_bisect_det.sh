mkdir -p gpurun_out/bis2
D="tests/test_gpu_production.py::test_deterministic_mode_bit_identical"
i=0
for grp in "tests/test_gpu_attention_ops.py tests/test_gpu_debug_build.py tests/test_gpu_decode.py tests/test_gpu_decode_parity.py" "tests/test_gpu_dist.py tests/test_gpu_frames.py tests/test_gpu_lstm.py" "tests/test_gpu_model.py tests/test_gpu_pipeline.py"; do
  i=$((i+1))
  timeout -k 10 400 python -u -m pytest $grp "$D" -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/bis2/g$i.log 2>&1
  echo "group $i [$grp]: $(tail -1 gpurun_out/bis2/g$i.log)"
done
