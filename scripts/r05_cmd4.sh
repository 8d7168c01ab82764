# round 5: config-3 walk occupancy A/B (shard and full batch)
TAG=r05occ WLS=config3 VARIANTS="base v6 v6c3" REPS="1 2" EXTRA="--queries 1024" SFX=_q1024 bash scripts/gpu_ab.sh && \
TAG=r05occ WLS=config3 VARIANTS="base v6c3" REPS="1" bash scripts/gpu_ab.sh
