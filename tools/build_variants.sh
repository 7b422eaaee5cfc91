# A/B builds of jh_lin.hip: tools/build_variants.sh name "-DFLAG ..." [name "flags"]...
set -e
cd "$(dirname "$0")/.."
python -c "from jepsen_amd import build as B; B.build_libjh()"
mkdir -p jepsen_amd/variants
while [ $# -ge 2 ]; do
  n=$1; f=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $f -c jepsen_amd/csrc/jh_lin.hip -o /tmp/jh_lin_$n.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o jepsen_amd/variants/libjh_$n.so /tmp/jh_lin_$n.o jepsen_amd/build/jh_counter.o jepsen_amd/build/jh_set.o jepsen_amd/build/jh_setfull.o jepsen_amd/build/jh_queue.o jepsen_amd/build/jh_api.o jepsen_amd/build/jh_multi.o jepsen_amd/build/jh_io.o jepsen_amd/build/jh_ingest.o -pthread
done
