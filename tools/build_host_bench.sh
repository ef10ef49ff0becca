# host-only build of tools/host_poseidon_bench.cpp with libtpst's host flags
# (baseline x86-64 ISA; TPST_HOST_ISA=v3 adds x86-64-v3 + ADX as build.py does)
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/bin
ISA=""
if [ "${TPST_HOST_ISA:-}" = "v3" ]; then ISA="-Xarch_host -march=x86-64-v3 -Xarch_host -madx"; fi
/opt/rocm/bin/hipcc -std=c++17 -O3 -x hip --offload-arch=gfx950 $ISA tools/host_poseidon_bench.cpp -o tools/bin/host_poseidon_bench
