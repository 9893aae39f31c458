# Diagnostic builds of libniti_hip.so with niti_wgrad.hip variants: tools/ablate/<name>/libniti_hip.so
# VARIANTS="st=-DNITI_WG_STAMPS=1 a1=-DNITI_WG_STAMPS=1,-DNITI_WG_ABLATE=1 ..."
set -e
cd "$(dirname "$0")/../mandheling-dsp-training_amd/csrc"
make -s
pids=""
for v in ${VARIANTS:-st=-DNITI_WG_STAMPS=1}; do
  name=${v%%=*}; flags=${v#*=}
  d=../../tools/ablate/$name
  mkdir -p $d
  ( /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC ${flags//,/ } -c niti_wgrad.hip -o $d/w.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $d/libniti_hip.so $d/w.o ../niti_amd/_lib/obj/niti_kernels.o ../niti_amd/_lib/obj/niti_resnet.o ../niti_amd/_lib/obj/niti_quant.o ../niti_amd/_lib/obj/niti_execution.o ../niti_amd/_lib/obj/niti_model.o ../niti_amd/_lib/obj/niti_capi.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib ) &
  pids="$pids $!"
done
for p in $pids; do wait $p; done
