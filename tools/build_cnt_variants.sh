# A/B builds of jh_counter.hip: tools/build_cnt_variants.sh name "-DFLAG ..." [name "flags"]...
set -e
cd "$(dirname "$0")/.."
python -c "from jepsen_amd import build as B; B.build_libjh()"
mkdir -p jepsen_amd/variants
while [ $# -ge 2 ]; do
  n=$1; f=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $f -c jepsen_amd/csrc/jh_counter.hip -o /tmp/jh_cnt_$n.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o jepsen_amd/variants/libjh_$n.so jepsen_amd/build/jh_lin.o /tmp/jh_cnt_$n.o jepsen_amd/build/jh_set.o jepsen_amd/build/jh_setfull.o jepsen_amd/build/jh_queue.o jepsen_amd/build/jh_api.o jepsen_amd/build/jh_multi.o jepsen_amd/build/jh_io.o jepsen_amd/build/jh_ingest.o -pthread
done
