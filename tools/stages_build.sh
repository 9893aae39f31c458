# Diagnostic builds of libniti_hip.so (timing only): tools/ablate/<name> for each NAME=FLAGS pair,
# e.g. VARIANTS="s8=-DNITI_TAPS_STAGES1=8 a5=-DNITI_ABLATE=5 nt=-DNITI_TAPS_NT=1".
set -e
cd "$(dirname "$0")/../mandheling-dsp-training_amd/csrc"
for v in ${VARIANTS:-s6=-DNITI_TAPS_STAGES1=6 s8=-DNITI_TAPS_STAGES1=8}; do
  name=${v%%=*}; flags=${v#*=}
  d=../../tools/ablate/$name
  mkdir -p $d
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC ${flags//,/ } -c niti_kernels.hip -o $d/k.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $d/libniti_hip.so $d/k.o ../niti_amd/_lib/obj/niti_quant.o ../niti_amd/_lib/obj/niti_execution.o ../niti_amd/_lib/obj/niti_model.o ../niti_amd/_lib/obj/niti_capi.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
done
