# Scheduler / agent / recommender image (one image, three entry points).
FROM rocm/pytorch:rocm7.0_ubuntu22.04_py3.10_pytorch_release_2.7.1
WORKDIR /opt/gpusched
COPY k8s_gpu_scheduler_amd/ k8s_gpu_scheduler_amd/
COPY native/ native/
COPY bench.py __graft_entry__.py ./
RUN pip install --no-cache-dir grpcio protobuf pyyaml scikit-learn prometheus_client pybind11 && \
    PYTORCH_ROCM_ARCH=gfx950 python3 -m k8s_gpu_scheduler_amd._native.build --force
ENV PYTHONPATH=/opt/gpusched
ENTRYPOINT ["python3", "-m", "k8s_gpu_scheduler_amd"]
