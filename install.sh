#!/bin/bash
# Install the MI355X GPU scheduler stack (recursive apply -- the reference's
# non-recursive `kubectl apply -f deploy` skipped the recommender).
set -euo pipefail
cd "$(dirname "$0")"
kubectl apply -f deploy/redis/redis-namespace.yaml
kubectl apply -f deploy/redis/
kubectl apply -f deploy/recommender/recommender-namespace.yaml
kubectl -n recommender create configmap recommender-data \
  --from-file=k8s_gpu_scheduler_amd/data/ --dry-run=client -o yaml | kubectl apply -f -
kubectl apply -f deploy/recommender/
kubectl apply -f deploy/profiler/
kubectl apply -f deploy/monitoring/
kubectl apply -f deploy/rbac.yaml -f deploy/scheduler.yaml
echo "installed; try: kubectl apply -f deploy/busybox/busybox.yaml"
