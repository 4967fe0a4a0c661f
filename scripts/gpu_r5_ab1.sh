OUT=r5_ab_c3 TESTS="-m gpu tests" bash scripts/gpu_ab.sh base startrsq cl cw4 cw2 && OUT=r5_ab_c4 BENCH_ARGS="--config c4" bash scripts/gpu_ab.sh base cw8
