C5="--scene s256 --depth 8 --spp 16 --steps 4 --warmup 2"
bash scripts/gpu_abv.sh c5 "base::$C5" "noshade:eraytracer_amd/variants/librtmi355x_noshade.so:$C5" "norefl:eraytracer_amd/variants/librtmi355x_norefl.so:$C5" && RT_LIB_PATH=$PWD/eraytracer_amd/variants/librtmi355x_stats.so timeout -k 10 200 python scripts/stats_run.py
