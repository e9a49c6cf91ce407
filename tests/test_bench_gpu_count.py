"""bench.visible_gpu_count counts GPUs from the KFD topology without
initialising HIP (the self-launching parent must not touch the GPU before its
rank children), narrowed by the *_VISIBLE_DEVICES variables."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _topology(tmp_path, gpu_ids):
    base = tmp_path / "nodes"
    for i, g in enumerate(gpu_ids):
        d = base / str(i)
        d.mkdir(parents=True)
        (d / "gpu_id").write_text("%d\n" % g)
    return str(base)


def test_counts_gpu_nodes_only(tmp_path):
    import bench
    nodes = _topology(tmp_path, [0, 0, 1234, 5678, 91011])  # two CPU nodes, three GPUs
    assert bench.visible_gpu_count(env={}, kfd_nodes=nodes) == 3


def test_visible_devices_narrow_the_count(tmp_path):
    import bench
    nodes = _topology(tmp_path, [0] + list(range(1, 9)))
    assert bench.visible_gpu_count(env={}, kfd_nodes=nodes) == 8
    assert bench.visible_gpu_count(env={"HIP_VISIBLE_DEVICES": "0,1"}, kfd_nodes=nodes) == 2
    assert bench.visible_gpu_count(env={"ROCR_VISIBLE_DEVICES": "3"}, kfd_nodes=nodes) == 1
    assert bench.visible_gpu_count(env={"CUDA_VISIBLE_DEVICES": ""}, kfd_nodes=nodes) == 0


def test_no_topology_means_no_gpu(tmp_path):
    import bench
    assert bench.visible_gpu_count(env={}, kfd_nodes=str(tmp_path / "absent")) == 0


def test_count_does_not_initialise_hip(tmp_path):
    import torch
    import bench
    bench.visible_gpu_count(env={}, kfd_nodes=_topology(tmp_path, [0, 7]))
    assert not torch.cuda.is_initialized()
