set -o pipefail
O=gpurun_out/x; rm -rf $O; mkdir -p $O
for i in 1 2; do
  DHTGPU_X_NOF4S=1 timeout -k 10 120 python bench.py --no-cpu --no-extra --no-scan --verify 0 > $O/nof4s_$i.log 2>&1
  echo "f4t-only $(grep timed $O/nof4s_$i.log)"
  timeout -k 10 120 python bench.py --no-cpu --no-extra --no-scan > $O/hint_$i.log 2>&1 || exit 1
  echo "f4t+small-f4 $(grep timed $O/hint_$i.log)"
done
