# k=11 bucket-kernel ablations (wrong counts by design; timing only), one process
timeout -k 10 400 python tools/lib_ab.py --libs kf2vecfsw_amd/libkf2vec_gpu.so,${ABL_LIBS:-tools/zoo/libkf2vec_abl3.so,tools/zoo/libkf2vec_abl4.so,tools/zoo/libkf2vec_abl5.so} --k 11 --rounds 3 --reps 4 > gpurun_out/abl_k11.json 2>&1; grep -A1 '\.so' gpurun_out/abl_k11.json
