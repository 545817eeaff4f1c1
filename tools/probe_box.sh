set -x
nproc; lscpu | grep -E "Model name|Socket|NUMA node\(s\)|Thread|Core"; free -g
ls /opt/conda/lib/libmkl_rt.so* ; ls /opt/rocm/lib/librocsparse.so*
rocm-smi --showproductname | head -20
python -c "import torch;print(torch.cuda.is_available(), torch.cuda.get_device_name(0))"
