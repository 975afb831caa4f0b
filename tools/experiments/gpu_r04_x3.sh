# K2: workgroups per CU and measurement builds (no table read / no histogram)
set -o pipefail
bash tools/experiments/gpu_k2_libs.sh r04x3 tree=tree p2=opendht_amd/ab/k2_p2.so p3=opendht_amd/ab/k2_p3.so p4=opendht_amd/ab/k2_p4.so m1=opendht_amd/ab/k2_p4m1.so m2=opendht_amd/ab/k2_p4m2.so m3=opendht_amd/ab/k2_p4m3.so > /dev/null || exit 1
echo ok
