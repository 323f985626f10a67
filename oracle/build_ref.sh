#!/usr/bin/env bash
# TEST INFRASTRUCTURE ONLY.  Builds oracle/_ref/ref_driver: the reference's hot-path
# Fortran compiled unmodified from /root/reference/src (read in place, never copied)
# plus oracle/ref_driver.F90.  Needs amdflang (ROCm) and MPICH (/opt/conda); runs only
# in the build container (the reference does not exist on the GPU box).
#
# Left out: amain.F90 / mod_time_loop.F90 (driver), mod_restart.F90 and
# diagnostics_nc.F90 (need netcdf-fortran, absent).  p4est (absent) is only referenced
# from mesh-construction routines that are never called; --gc-sections drops them.
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
SRC="${HNUMO_REF_SRC:-/root/reference/src}"
OUT="$HERE/_ref"
OBJ="$OUT/obj"
FC="${FC:-/opt/rocm/lib/llvm/bin/amdflang}"
MPI_INC=/opt/conda/include
MPI_LIB=/opt/conda/lib
# -fdefault-real-8: the reference's own build flag (config.user:25,61)
FLAGS="-O2 -fdefault-real-8 -cpp -D__PGI"
[ -d "$SRC" ] || { echo "reference sources not found at $SRC" >&2; exit 2; }
mkdir -p "$OBJ"
cd "$OBJ"
EXCLUDE="amain.F90 mod_time_loop.F90 mod_restart.F90 diagnostics_nc.F90"
$FC $FLAGS -I"$MPI_INC" -c "$HERE/mpi_module.F90" -o mpi_module.o
files=""
for f in $(cd "$SRC" && ls *.F90); do
  case " $EXCLUDE " in *" $f "*) continue;; esac
  files="$files $f"
done
for pass in $(seq 1 15); do
  left=0
  for f in $files; do
    o="${f%.F90}.o"
    [ -f "$o" ] && [ "$o" -nt "$SRC/$f" ] && continue
    if ! $FC $FLAGS -I. -c "$SRC/$f" -o "$o" 2>"${f%.F90}.err"; then left=$((left+1)); rm -f "$o"; fi
  done
  [ $left -eq 0 ] && break
done
if [ $left -ne 0 ]; then
  echo "reference build failed; see $OBJ/*.err" >&2; exit 1
fi
$FC $FLAGS -I. -c "$HERE/ref_driver.F90" -o ref_driver.o
# -finit-real=zero for the one never-assigned automatic array the path reads (zero_init_wrap.c)
gcc -O2 -c "$HERE/zero_init_wrap.c" -o zero_init_wrap.o
WRAP="-Wl,--wrap=_QMmod_create_rhs_mlswePrhs_layer_shear_stress"
REFOBJ=$(ls *.o | grep -v -e '^ref_driver.o$' -e '^dropin_driver.o$' -e '^hnumo_' -e '^zero_init_wrap.o$')
$FC -O2 -o "$OUT/ref_driver" ref_driver.o zero_init_wrap.o $REFOBJ $WRAP \
    -L"$MPI_LIB" -Wl,-rpath,"$MPI_LIB" -lmpifort -lmpi -Wl,--gc-sections
echo "built $OUT/ref_driver"

# The drop-in: the same harness with ti_rk_bcl replaced by the Fortran bridge to the HIP
# engine (include/hnumo_engine.f90 + h-numo_amd/fortran/hnumo_bridge.F90).  Runs on a GPU.
REPO="$(cd "$HERE/.." && pwd)"
ENGINE="$REPO/h-numo_amd/libhnumo_engine.so"
if [ -f "$ENGINE" ]; then
  $FC $FLAGS -I. -c "$REPO/include/hnumo_engine.f90" -o hnumo_engine_f.o
  $FC $FLAGS -I. -c "$REPO/h-numo_amd/fortran/hnumo_bridge.F90" -o hnumo_bridge.o
  $FC $FLAGS -DHNUMO_DROPIN -I. -c "$HERE/ref_driver.F90" -o dropin_driver.o
  $FC -O2 -o "$OUT/dropin_driver" dropin_driver.o hnumo_bridge.o hnumo_engine_f.o zero_init_wrap.o $REFOBJ $WRAP \
      -L"$REPO/h-numo_amd" -Wl,-rpath,'$ORIGIN/../../h-numo_amd' -lhnumo_engine \
      -L"$MPI_LIB" -Wl,-rpath,"$MPI_LIB" -lmpifort -lmpi -Wl,--gc-sections
  echo "built $OUT/dropin_driver"
fi
