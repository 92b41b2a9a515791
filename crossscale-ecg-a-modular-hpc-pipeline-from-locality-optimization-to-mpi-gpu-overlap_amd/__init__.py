"""CrossScale-ECG for MI355X.

An MI355X-native (gfx950 / CDNA4) re-design of the three-module CrossScale-ECG study
(reference: sm-edwards/CrossScale-ECG-A-Modular-HPC-Pipeline-from-Locality-Optimization-to-MPI-GPU-Overlap):

* Module 1 (data locality)  -> ``data``   : binary ECG shards, C++ mmap reader, hipHostMalloc pinned ring,
                                             copy-stream H2D, GPU-resident shards sized for 288 GB HBM.
* Module 2 (conv1d kernel)  -> ``ops``    : hand-written HIP conv1d kernels (valid single-channel,
                                             multi-channel MFMA implicit GEMM) + C++ OpenMP/AVX CPU twin.
* Module 3 (federated)      -> ``parallel`` / ``train`` : FedAvg over RCCL (torch.distributed "nccl"),
                                             one FL client per GPU, fused single-kernel TinyECG step
                                             replayed from a HIP graph, comm/compute overlap.

Import as ``crossscale_ecg`` (see ``crossscale_ecg/__init__.py``).
"""

__version__ = "0.1.0"

# Parameter layout constants of TinyECG (reference Module_3/tiny_ecg_model.py:16-23).
HIDDEN_CHANNELS = 16
CONV1_KERNEL = 7
CONV2_KERNEL = 5
DEFAULT_WINDOW = 500
