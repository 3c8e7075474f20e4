C2="--scene default --width 1920 --height 1080 --depth 5 --no-cpu-baseline --no-boundary --no-setup"
for rep in 1 2; do
for v in "base:" "wave:RT_ENGINE=wave" "if6:--inflight 6" "if8:--inflight 8" "if3:--inflight 3"; do
  name=${v%%:*}; a=${v#*:}; envs=""; args=""
  case $a in RT_*) envs=$a;; *) args=$a;; esac
  env $envs timeout -k 10 200 python bench.py $C2 $args > gpurun_out/c2ab_one.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['config']['engine'])" gpurun_out/c2ab_one.json "$name rep$rep" | tee -a gpurun_out/r06l_c2_ab.txt
done; done
