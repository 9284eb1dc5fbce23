W="--steps 256 --warmup 64 --no-cpu-baseline"
export PLAN="R1_64k_run_trio||--workload R1 --n-envs 65536 --nstep-pop running --schedule trio $W
R1_64k_run_single||--workload R1 --n-envs 65536 --nstep-pop running --schedule single $W
R1_32k_run_trio||--workload R1 --n-envs 32768 --nstep-pop running --schedule trio $W
R1_32k_run_single||--workload R1 --n-envs 32768 --nstep-pop running --schedule single $W
R1_64k_exact_trio||--workload R1 --n-envs 65536 --schedule trio $W
R1_64k_run_trio2||--workload R1 --n-envs 65536 --nstep-pop running --schedule trio $W
R1_64k_run_single2||--workload R1 --n-envs 65536 --nstep-pop running --schedule single $W"
export TAG=r06p
bash tools/ab_bench.sh
