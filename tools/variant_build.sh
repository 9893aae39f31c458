# Diagnostic variant builds of libniti_hip.so: tools/ablate/<name>/libniti_hip.so built with
# extra defines.  Usage: bash tools/variant_build.sh name "-DFOO=1 -DBAR=2" [name2 "defs2" ...]
set -e
cd "$(dirname "$0")/../mandheling-dsp-training_amd/csrc"
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  mkdir -p ../../tools/ablate/$name
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC $defs -c niti_kernels.hip -o ../../tools/ablate/$name/k.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../../tools/ablate/$name/libniti_hip.so ../../tools/ablate/$name/k.o ../niti_amd/_lib/obj/niti_execution.o ../niti_amd/_lib/obj/niti_model.o ../niti_amd/_lib/obj/niti_capi.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
done
