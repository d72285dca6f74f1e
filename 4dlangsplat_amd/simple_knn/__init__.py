"""simple_knn -- drop-in for the un-vendored submodule submodules/simple-knn
(/root/reference/.gitmodules:1-3), backed by liblsr.so (include/lsr_knn.h, knn.hip).

The reference imports it at scene/gaussian_model.py:22 (`from simple_knn._C import distCUDA2`)
and calls it once per scene initialisation (scene/gaussian_model.py:203-204).
"""
