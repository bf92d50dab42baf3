# same-box A/B of library builds (tools/build_variant.sh): the default
# library against build_var/libabc_<name>.so for each name in AB_LIBS
# ("a+b"), interleaved, per shape in AB_SHAPES ("N/d+N/d", or "N/d/M" for
# M new rows against N); rows compared by checksum (tools/kde_time.py)
set -e
out=gpurun_out/${AB_NAME:-ab}/ab.txt
IFS='+' read -ra shapes <<< "${AB_SHAPES:-1e6/8}"
IFS='+' read -ra libs <<< "${AB_LIBS}"
for shape in "${shapes[@]}"; do
  for rep in 1 2; do
    for lib in pyabc_amd/_lib/libabc_hip.so "${libs[@]}"; do
      case $lib in */*) ;; *) lib=build_var/libabc_$lib.so ;; esac
      IFS='/' read -r n dd m <<< "$shape"
      timeout -k 10 120 python3 -u tools/lib_ab.py "$lib" tools/kde_time.py \
        "$n" "$dd" 7 - "${m:-$n}" >> "$out" 2>/dev/null
    done
  done
done
