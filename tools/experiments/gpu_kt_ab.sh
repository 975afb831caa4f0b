# pipelined kernel traces (rocprofv3 --kernel-trace) of HEAD and the old_r02 worktree, same box
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ktab; rm -rf $O; mkdir -p $O
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/head -o run --output-format csv -- python3 bench.py --no-scan --no-cpu --no-extra --steps 300 --warmup 20 > $O/head.log 2>&1 || exit 1
(cd old_r02 && timeout -k 10 180 rocprofv3 --kernel-trace -d ../$O/old -o run --output-format csv -- python3 bench.py --no-scan --no-cpu --no-extra --steps 300 --warmup 20) > $O/old.log 2>&1 || exit 1
python3 tools/kt_pipe_cmp.py $O/head $O/old
