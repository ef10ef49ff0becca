# host-only build of tools/host_poseidon_bench.cpp with libtpst's host flags
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/bin
/opt/rocm/bin/hipcc -std=c++17 -O3 -x hip --offload-arch=gfx950 -Xarch_host -march=x86-64-v3 -Xarch_host -madx \
  tools/host_poseidon_bench.cpp -o tools/bin/host_poseidon_bench
