! TEST INFRASTRUCTURE ONLY (oracle/_ref build).  MPICH (/opt/conda) ships its `mpi`
! Fortran module only as a gfortran .mod file, which flang cannot read.  This compiles
! the same module for flang from MPICH's own mpif.h; the library linked is MPICH itself.
module mpi
include "mpif.h"
end module mpi
