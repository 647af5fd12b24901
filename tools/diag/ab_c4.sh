B="python bench.py --config c4 --steps 4 --warmup 1 --no-cpu-baseline --no-config1 --first-steps 0"
tools/gpu_steps.sh "base1|120|$B" "lazy1|120|IRLMX_LIB=build/lazy/libirlmx.so $B" "base2|120|$B" "lazy2|120|IRLMX_LIB=build/lazy/libirlmx.so $B"
