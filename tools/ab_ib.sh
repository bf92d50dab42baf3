# same-box A/B of the d <= 8 i-block build option (tools/build_variant.sh
# ib4 "-DABC_KDE_IB_SMALL=4"): the default library against the variant,
# interleaved, per shape; rows compared by checksum (tools/kde_time.py)
set -e
out=gpurun_out/${AB_NAME:-ab}/ab.txt
for shape in "1e6 8" "1e6 4" "1e5 4" "1e6 6" "1e6 2" "2e5 8"; do
  for rep in 1 2; do
    for lib in pyabc_amd/_lib/libabc_hip.so build_var/libabc_ib4.so; do
      timeout -k 10 120 python3 -u tools/lib_ab.py $lib tools/kde_time.py $shape 5 >> $out 2>/dev/null
    done
  done
done
for rep in 1 2; do
  ABC_KDE_MFMA_LDS2=2 timeout -k 10 120 python3 -u tools/lib_ab.py build_var/libabc_ib4.so tools/kde_time.py 1e6 8 5 ib4_pipelined >> $out 2>/dev/null
done
