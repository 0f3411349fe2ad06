for E in 2; do echo "== exp $E"; RTREC_HIP_LIB=$PWD/exp/librtrec_e$E.so timeout -k 10 200 python -u tools/microbench_topk.py 2>&1 | grep -v amdgpu.ids | grep float16 | head -3; done
bash tools/_gpu_tb.sh
