H="MADIGAN_LIB_PATH=tools/_var/head/libmadigan_hip.so"
N20="--nstep 20 --nstep-pop running --steps 20 --warmup 5 --fuse 20 --no-k-sweep"
W="--steps 128 --warmup 64"
export TAG=r06f
export PLAN="n20_head|$H|$N20
n20_cur||$N20
n20_head2|$H|$N20
n20_cur2||$N20
R1_64k_head|$H|--workload R1 --n-envs 65536 $W
R1_64k_cur||--workload R1 --n-envs 65536 $W
R1_64k_eg1|MGN_GATHER_EG=1|--workload R1 --n-envs 65536 $W
R1_64k_eg4|MGN_GATHER_EG=4|--workload R1 --n-envs 65536 $W
R1_64k_nolds|MGN_GATHER_LDS=0|--workload R1 --n-envs 65536 $W
R1_64k_eg4_nolds|MGN_GATHER_EG=4 MGN_GATHER_LDS=0|--workload R1 --n-envs 65536 $W
R1_64k_eg1_nolds|MGN_GATHER_EG=1 MGN_GATHER_LDS=0|--workload R1 --n-envs 65536 $W
R1_8k_head|$H|--workload R1 --n-envs 8192 $W
R1_8k_cur||--workload R1 --n-envs 8192 $W
C5_head|$H|--workload C5 $W
C5_cur||--workload C5 $W
C5_nolds|MGN_GATHER_LDS=0|--workload C5 $W
C2_head|$H|--workload C2 $W
C2_cur||--workload C2 $W
C2_eg1|MGN_GATHER_EG=1|--workload C2 $W
C2_nolds|MGN_GATHER_LDS=0|--workload C2 $W
C4_head|$H|--workload C4 $W
C4_cur||--workload C4 $W
C4_eg1|MGN_GATHER_EG=1|--workload C4 $W"
bash tools/ab_bench.sh
