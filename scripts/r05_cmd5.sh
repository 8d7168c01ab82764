# round 5: XCD-aligned walk task mapping A/B
TAG=r05xcd WLS=config3 VARIANTS="base xcdwalk" REPS="1 2" EXTRA="--queries 1024" SFX=_q1024 bash scripts/gpu_ab.sh && \
TAG=r05xcd WLS="config3 config2" VARIANTS="base xcdwalk" REPS="1" EXTRA="--no-size-sweep" bash scripts/gpu_ab.sh
