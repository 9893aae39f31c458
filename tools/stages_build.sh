# Diagnostic builds of libniti_hip.so (timing only, results may be wrong by design): one source
# file rebuilt with extra flags, linked with the other objects of the in-tree build, into
# tools/ablate/<name>/libniti_hip.so for each NAME=FLAGS pair (commas become spaces), e.g.
#   SRC=niti_rowconv.hip VARIANTS="e1=-DRC_EXP=1 e4=-DRC_EXP=4" tools/stages_build.sh
#   SRC=niti_kernels.hip VARIANTS="s8=-DNITI_TAPS_STAGES1=8" tools/stages_build.sh
# Select one at run time with NITI_HIP_LIB=tools/ablate/<name>/libniti_hip.so.
set -e
cd "$(dirname "$0")/../mandheling-dsp-training_amd/csrc"
make -s
SRC=${SRC:-niti_rowconv.hip}
OBJ=../niti_amd/_lib/obj
others=$(ls $OBJ/*.o | grep -v "/${SRC%.hip}.o$")
for v in ${VARIANTS:?set VARIANTS=\"name=flags ...\"}; do
  name=${v%%=*}; flags=${v#*=}
  d=../../tools/ablate/$name
  mkdir -p $d
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -w ${flags//,/ } -c $SRC -o $d/v.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $d/libniti_hip.so $d/v.o $others -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
done
