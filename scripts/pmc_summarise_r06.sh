#!/bin/bash
# Summaries of gpu_prof_r06.sh's counter passes into profiles/ (run here, after
# the GPU call merged gpurun_out/TAG back):  bash scripts/pmc_summarise_r06.sh TAG
set -e
O=gpurun_out/${1:-r06p}
export LZ_COMMIT=$(git rev-parse --short HEAD)
python scripts/pmc_traffic.py $O/fetch_c3 $O/write_c3 "k_wf16<11,1936,3,1,4,1,true,false,false,0>" k_wf16 10000000 100000182 4096 profiles/r06_pmc_k_wf16.json "k_wf16<11,1936,3,1,4,1,true,false,false,1>"
python scripts/pmc_traffic.py $O/fetch_c3 $O/write_c3 "k_spmm_seg<double,16,48,768,false,0,false,false,false>" k_spmm_seg 10000000 100000182 4096 profiles/r06_pmc_k_spmm_seg.json
python scripts/pmc_traffic.py $O/fetch_c4r $O/write_c4r "k_wf16<10,4400,2,1,2,1,false,false,false,0>" k_wf16 5000000 124909886 65536 profiles/r06_c4rank_pmc_k_wf16.json
python scripts/pmc_traffic.py $O/fetch_c5 $O/write_c5 "k_spmm_seg<float,32,48,1024,false,0,false,true,false>" k_spmm_seg_c5 10000000 99393762 0 profiles/r06_pmc_k_spmm_seg_c5.json
python scripts/pmc_traffic.py $O/fetch_rand $O/write_rand "k_spmm_seg<double,16,48,768,false,0,false,false,false>" k_spmm_seg_random_columns 10000000 95333504 10000000 profiles/r06_pmc_k_spmm_seg_random_columns.json
python scripts/pmc_mfma.py $O/mfma_c3 r06 10000000 100000182 4096 "k_wf16<11,1936,3,1,4,1,true,false,false,0>"
python scripts/pmc_mfma.py $O/mfma_c4r r06_c4rank 5000000 124909886 65536 "k_wf16<10,4400,2,1,2,1,false,false,false,0>"
cp $O/trace_c3/run_kernel_stats.csv profiles/r06_kernel_stats.csv 2>/dev/null || find $O/trace_c3 -name "*kernel_stats.csv" -exec cp {} profiles/r06_kernel_stats.csv \;
find $O/trace_c4r -name "*kernel_stats.csv" -exec cp {} profiles/r06_c4r_kernel_stats.csv \;
cp $O/gaps_c3.txt profiles/r06_kernel_gaps.txt
cp $O/bench_c4rank.json profiles/r06_bench_c4rank.json
