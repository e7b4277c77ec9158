# register / spill / LDS report of the kernels in one translation unit: bash tools/res.sh FILE.hip [PATTERN] [EXTRA FLAGS...]
f=${1:?file}; pat=${2:-.}; shift; shift
cd nice-slam_amd/csrc && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -munsafe-fp-atomics \
  -I../../include -Wall -Wno-unused-function "$@" -c $f -o /tmp/res_$$.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk -v pat="$pat" '/Function Name/ {show = ($0 ~ pat); if (show) print $NF " " $(NF-1)} show && /VGPRs:|AGPRs|Spill|LDS Size|Occupancy/ {sub(/.*remark: +/, "  "); sub(/ \[-Rpass.*/, ""); print}'
rm -f /tmp/res_$$.o
