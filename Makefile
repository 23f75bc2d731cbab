# Build / test / run targets (the reference's Makefile builds a Go binary + images).
PY ?= python3
IMAGE ?= gpusched/gpu-scheduler-rocm
TAG ?= 0.1.0

.PHONY: native native-asan test test-gpu bench profile-tables image push deploy clean

native:
	$(PY) -m k8s_gpu_scheduler_amd._native.build

native-asan:                 ## host modules with -fsanitize=address,undefined
	$(PY) -m k8s_gpu_scheduler_amd._native.build --asan --only _core _smi

test: native
	$(PY) -m pytest tests -m "not gpu" -q

test-gpu: native
	$(PY) -m pytest tests -m gpu -q

bench: native
	$(PY) bench.py --steps 20 --warmup 3

profile-tables: native
	$(PY) -m k8s_gpu_scheduler_amd.models.profile

image:
	docker build -t $(IMAGE):$(TAG) .

push: image
	docker push $(IMAGE):$(TAG)

deploy:
	./install.sh

clean:
	rm -f k8s_gpu_scheduler_amd/_native/*.so
