# build a variant library: variant.sh NAME "EXTRA FLAGS"
set -e
cd /root/repo/partisan_amd/csrc
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-label -Wno-unused-value -Wno-unused-result"
/opt/rocm/bin/hipcc $F $2 -c psim_consume.hip -o /tmp/pc_$1.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o libpartisan_gpu_sim_$1.so /tmp/pc_$1.o psim_strategy.o psim_engine.o -L/opt/rocm/lib -lrccl
