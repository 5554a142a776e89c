set -x
which ffmpeg ffprobe || true
ls /usr/lib/x86_64-linux-gnu | grep -i -E "avcodec|swscale|jpeg" || true
nproc; lscpu | grep -E "Model name|^CPU\(s\)|Thread|Socket" || true
rocm-smi --showproductname || true
timeout -k 10 120 python -c "import torch;print(torch.cuda.is_available(), torch.cuda.get_device_name(0), torch.cuda.get_device_properties(0))"
free -g
