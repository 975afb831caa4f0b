# Round 5, pass t: which part of F3's hand-off of w0 ties to F4 costs F3 its ~4 us (one-set cfg 2,
# every build handing ties to F4: deferall = the pre-inline form; without the candidate copy,
# without the header store, without both; noties = no tie handling at all).  F3/F4 event times.
set -o pipefail
OUT=gpurun_out/r05t; mkdir -p $OUT
for i in 1 2; do
  for v in tree deferall defnocopy defnohdr defnone noties; do
    lib=""; [ $v != tree ] && lib=opendht_amd/ab/$v.so
    echo -n "$v "; DHTGPU_LIB=$lib timeout -k 10 120 python tools/batch_probe.py --reps 20 2>&1 | grep "phases ms" || exit 1
  done
done | tee $OUT/defer_bisect.txt
