# Host-side AddressSanitizer check of libnslam.so (CPU container; GPU ASan is not available on the
# pool): the library's host code built with -fsanitize=address (device code unchanged), loaded into
# the CPU test process with the clang ASan runtime preloaded, running every argument-validation and
# struct-layout path of tests/test_abi_cpu.py.  usage: bash tools/asan_host.sh
set -euo pipefail
cd "$(dirname "$0")/.."
make -C nice-slam_amd/csrc -j8 variant V=asan X="-Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer" > /tmp/asan_build.log 2>&1
mkdir -p /tmp/nslam_asan && mv nice-slam_amd/libnslam_asan.so /tmp/nslam_asan/   # keep it out of the GPU snapshot
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
echo "asan symbols: $(nm -D /tmp/nslam_asan/libnslam_asan.so | grep -c __asan)"
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 LD_PRELOAD=$RT NSLAM_LIB=/tmp/nslam_asan/libnslam_asan.so \
  python -m pytest tests/test_abi_cpu.py -q -p no:cacheprovider
