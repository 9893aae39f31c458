# Diagnostic builds of libniti_hip.so with parts of the GEMM loop removed (NITI_ABLATE=1: no
# global->LDS copies, 2: no MFMA).  Results are wrong by design; for timing only.
set -e
cd "$(dirname "$0")/../mandheling-dsp-training_amd/csrc"
for v in 1 2 3 4; do
  mkdir -p ../../tools/ablate/$v
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -DNITI_ABLATE=$v -c niti_kernels.hip -o ../../tools/ablate/$v/k.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../../tools/ablate/$v/libniti_hip.so ../../tools/ablate/$v/k.o ../niti_amd/_lib/obj/niti_execution.o ../niti_amd/_lib/obj/niti_model.o ../niti_amd/_lib/obj/niti_capi.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
done
