# Host-side AddressSanitizer + UBSan build of the native library's CPU code and its driver (tests/asan/host_main.cpp).
# Device code is compiled as usual; -fsanitize applies to the host pass only (-Xarch_host, as the pool requires).
# Runs on the CPU (no kernel launch).   bash tools/asan_host.sh  -> build/asan/host_main, then runs it.
set -e
cd "$(dirname "$0")/.."
OUT=build/asan
mkdir -p $OUT
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer"
FLAGS="-O1 -g -std=c++17 -fPIC --offload-arch=gfx950 -Ighost_amd/csrc -Iinclude"
pids=""
for f in ghost_amd/csrc/*.hip; do
  o=$OUT/$(basename ${f%.hip}).o
  if [ ! -f $o ] || [ $f -nt $o ] || [ -n "$(find ghost_amd/csrc include -name '*.h' -newer $o)" ]; then
    /opt/rocm/bin/hipcc $FLAGS $SAN -c $f -o $o &
    pids="$pids $!"
  fi
done
for p in $pids; do wait $p; done
/opt/rocm/bin/hipcc $FLAGS $SAN -c tests/asan/host_main.cpp -o $OUT/host_main.obj
/opt/rocm/bin/hipcc --offload-arch=gfx950 $SAN $OUT/host_main.obj $OUT/*.o -o $OUT/host_main
ASAN_OPTIONS=detect_leaks=1:abort_on_error=0 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 $OUT/host_main
