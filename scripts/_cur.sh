export ROUND=r6
L=humanoid_mppi-rl_amd/lib
bash scripts/gpu_pass.sh tests s4 "x3d or config4_full_size_matches_oracle or horizon_tails or probe" &&
bash scripts/gpu_pass.sh ab s4 x3d8 "--workload humanoid_ca --global-solves 8" - $L/libmppi_hip_prev.so -,MPPI_X3D=0 - $L/libmppi_hip_prev.so -,MPPI_X3D=0 &&
bash scripts/gpu_pass.sh ab s4 x3d16 "--workload humanoid_ca --global-solves 16" - -,MPPI_X3D=0
