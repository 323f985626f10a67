! hnumo_engine.f90 -- Fortran ISO_C_BINDING interface to libhnumo_engine (include/hnumo_engine.h).
!
! The derived types mirror the C descriptor structs field for field (same order, bind(C)
! layout); every array field is a type(c_ptr) to the caller's Fortran array.  The engine
! copies everything it needs during hnumo_engine_create, so the descriptors only have to
! stay valid for that call.  State arrays are passed by reference as assumed-size arrays.
!
! Build: amdflang -c include/hnumo_engine.f90   (any Fortran 2008 compiler).
! Link:  -L<repo>/h-numo_amd -lhnumo_engine -Wl,-rpath,<repo>/h-numo_amd
module hnumo_engine_c
    use iso_c_binding, only: c_int, c_int32_t, c_int64_t, c_double, c_ptr, c_char, c_null_ptr, &
        c_null_char, c_f_pointer, c_loc
    implicit none
    private

    integer(c_int), parameter, public :: HNUMO_OK = 0, HNUMO_ERR_NEGATIVE_THICKNESS = 1, &
        HNUMO_ERR_NONFINITE = 2, HNUMO_ERR_DEVICE = 3, HNUMO_ERR_INVALID = 4
    integer(c_int32_t), parameter, public :: HNUMO_SHEAR_CORRECTOR_REFERENCE = 0, &
        HNUMO_SHEAR_CORRECTOR_PREDICTED = 1
    integer(c_int), parameter, public :: HNUMO_ABI_EXPECTED = 10   ! must equal hnumo_abi_version()
    integer(c_int), parameter, public :: HNUMO_SUM_REFERENCE = 0, HNUMO_SUM_FACTORED = 1

    ! = hnumo_mesh_desc (mod_grid, mod_face, mod_basis, mod_metrics; optional dense tables)
    type, bind(C), public :: hnumo_mesh_desc
        integer(c_int32_t) :: nelem = 0, npoin = 0, npoin_q = 0, nface = 0
        integer(c_int32_t) :: ngl = 0, nq = 0, nlayers = 0
        type(c_ptr) :: face = c_null_ptr                       ! (8,nface)
        type(c_ptr) :: imapl = c_null_ptr, imapr = c_null_ptr ! (3,ngl,nface) = imapl(:,:,1,:)
        type(c_ptr) :: normal_vector = c_null_ptr             ! (3,ngl,nface)
        type(c_ptr) :: normal_vector_q = c_null_ptr           ! (3,nq,nface)
        type(c_ptr) :: jac_face = c_null_ptr                  ! (ngl,nface)
        type(c_ptr) :: jac_faceq = c_null_ptr                 ! (nq,nface)
        type(c_ptr) :: massinv = c_null_ptr                   ! (npoin)
        type(c_ptr) :: psiq = c_null_ptr, dpsiq = c_null_ptr  ! (ngl,nq)
        type(c_ptr) :: psi = c_null_ptr, dpsi = c_null_ptr    ! (ngl,ngl)
        type(c_ptr) :: ksiq_x = c_null_ptr, ksiq_y = c_null_ptr, etaq_x = c_null_ptr, &
            etaq_y = c_null_ptr, jacq = c_null_ptr            ! (nq,nq,nelem)
        type(c_ptr) :: ksi_x = c_null_ptr, ksi_y = c_null_ptr, eta_x = c_null_ptr, &
            eta_y = c_null_ptr, jac = c_null_ptr              ! (ngl,ngl,nelem)
        type(c_ptr) :: psih = c_null_ptr, dpsidx = c_null_ptr, dpsidy = c_null_ptr, wjac = c_null_ptr
        type(c_ptr) :: indexq = c_null_ptr
        type(c_ptr) :: dpsidx_df = c_null_ptr, dpsidy_df = c_null_ptr, wjac_df = c_null_ptr
        type(c_ptr) :: index_df = c_null_ptr
        type(c_ptr) :: imapl_q = c_null_ptr, imapr_q = c_null_ptr ! (3,nq,nface), method_visc == 1
    end type hnumo_mesh_desc

    ! = hnumo_static_desc (mod_initial.F90:42-53)
    type, bind(C), public :: hnumo_static_desc
        type(c_ptr) :: pbprime = c_null_ptr, pbprime_df = c_null_ptr
        type(c_ptr) :: one_over_pbprime = c_null_ptr, one_over_pbprime_df = c_null_ptr
        type(c_ptr) :: pbprime_face = c_null_ptr, pbprime_df_face = c_null_ptr
        type(c_ptr) :: one_over_pbprime_edge = c_null_ptr
        type(c_ptr) :: coeff_pbpert_L = c_null_ptr, coeff_pbpert_R = c_null_ptr, coeff_pbub_LR = c_null_ptr
        type(c_ptr) :: coeff_mass_pbub_L = c_null_ptr, coeff_mass_pbub_R = c_null_ptr, &
            coeff_mass_pbpert_LR = c_null_ptr
        type(c_ptr) :: alpha = c_null_ptr
        type(c_ptr) :: tau_wind = c_null_ptr, coriolis_quad = c_null_ptr, grad_zbot_quad = c_null_ptr
        type(c_ptr) :: zbot_df = c_null_ptr, zbot_face = c_null_ptr
        type(c_ptr) :: fdt2_bcl = c_null_ptr, a_bcl = c_null_ptr, b_bcl = c_null_ptr
        type(c_ptr) :: ssprk_a = c_null_ptr, ssprk_beta = c_null_ptr
    end type hnumo_static_desc

    ! = hnumo_params (mod_input, mod_constants, mod_initial N_btp)
    type, bind(C), public :: hnumo_params
        real(c_double) :: dt = 0, dt_btp = 0
        real(c_double) :: visc_mlswe = 0, cd_mlswe = 0, ad_mlswe = 0, gravity = 0
        integer(c_int32_t) :: N_btp = 0, kstages = 0, method_visc = 0, botfr = 0
        real(c_double) :: max_shear_dz = 0
        integer(c_int32_t) :: shear_corrector = 0, reserved = 0
    end type hnumo_params

    ! = hnumo_halo_desc (mod_parallel)
    type, bind(C), public :: hnumo_halo_desc
        integer(c_int32_t) :: rank = 0, nranks = 1, num_nbh = 0
        type(c_ptr) :: nbh_proc = c_null_ptr, num_send_recv = c_null_ptr, nbh_send_recv = c_null_ptr
        type(c_ptr) :: comm_id = c_null_ptr
        integer(c_int32_t) :: nelem_owned = 0
        type(c_ptr) :: num_ghost_send = c_null_ptr, ghost_send = c_null_ptr
        type(c_ptr) :: num_ghost_recv = c_null_ptr, ghost_recv = c_null_ptr
    end type hnumo_halo_desc

    public :: hnumo_engine_create, hnumo_engine_destroy, hnumo_abi_version, hnumo_ti_rk_bcl, &
        hnumo_ti_barotropic_ssprk, hnumo_btp_bcl_coeffs, hnumo_create_rhs_btp, hnumo_get_field_c, &
        hnumo_set_resident, hnumo_sync, hnumo_last_error_c, hnumo_last_error, hnumo_get_field, &
        hnumo_set_summation, hnumo_get_summation, hnumo_stage_path, hnumo_persistent_info, hnumo_predict, &
        hnumo_rccl_unique_id, hnumo_persistent_stats

    interface
        integer(c_int) function hnumo_engine_create(mesh, statics, params, halo, device, eng) &
                bind(C, name='hnumo_engine_create')
            import :: c_int, c_ptr, hnumo_mesh_desc, hnumo_static_desc, hnumo_params
            type(hnumo_mesh_desc), intent(in) :: mesh
            type(hnumo_static_desc), intent(in) :: statics
            type(hnumo_params), intent(in) :: params
            type(c_ptr), value :: halo                    ! hnumo_halo_desc* or c_null_ptr
            integer(c_int), value :: device
            type(c_ptr), intent(out) :: eng
        end function hnumo_engine_create

        subroutine hnumo_engine_destroy(eng) bind(C, name='hnumo_engine_destroy')
            import :: c_ptr
            type(c_ptr), value :: eng
        end subroutine hnumo_engine_destroy

        integer(c_int) function hnumo_abi_version() bind(C, name='hnumo_abi_version')
            import :: c_int
        end function hnumo_abi_version

        ! 128-byte RCCL unique id for hnumo_halo_desc%comm_id (made on one rank, broadcast)
        integer(c_int) function hnumo_rccl_unique_id(out128) bind(C, name='hnumo_rccl_unique_id')
            import :: c_int, c_char
            character(kind=c_char), intent(out) :: out128(128)
        end function hnumo_rccl_unique_id

        type(c_ptr) function hnumo_last_error_c(eng) bind(C, name='hnumo_last_error')
            import :: c_ptr
            type(c_ptr), value :: eng
        end function hnumo_last_error_c

        ! = ti_rk_bcl(q_df, qb_df, qprime_df)  (ti_rk_bcl.F90:9-87)
        integer(c_int) function hnumo_ti_rk_bcl(eng, q_df, qb_df, qprime_df) bind(C, name='hnumo_ti_rk_bcl')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: eng
            real(c_double), intent(inout) :: q_df(*), qb_df(*), qprime_df(*)
        end function hnumo_ti_rk_bcl

        ! = ti_barotropic_ssprk_mlswe(qb_df, qprime_df)  (mod_rk_mlswe.F90:19-151)
        integer(c_int) function hnumo_ti_barotropic_ssprk(eng, qb_df, qprime_df) &
                bind(C, name='hnumo_ti_barotropic_ssprk')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: eng
            real(c_double), intent(inout) :: qb_df(*)
            real(c_double), intent(in) :: qprime_df(*)
        end function hnumo_ti_barotropic_ssprk

        ! = btp_bcl_coeffs_qdf after extract_qprime_df_face  (ti_rk_bcl.F90:43-50)
        integer(c_int) function hnumo_btp_bcl_coeffs(eng, qprime_df) bind(C, name='hnumo_btp_bcl_coeffs')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: eng
            real(c_double), intent(in) :: qprime_df(*)
        end function hnumo_btp_bcl_coeffs

        ! = create_rhs_btp(rhs, qb_df, qprime_df)  (mod_rhs_btp.F90:28-59)
        integer(c_int) function hnumo_create_rhs_btp(eng, rhs, qb_df, qprime_df) bind(C, name='hnumo_create_rhs_btp')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: eng
            real(c_double), intent(out) :: rhs(*)
            real(c_double), intent(in) :: qb_df(*), qprime_df(*)
        end function hnumo_create_rhs_btp

        integer(c_int) function hnumo_get_field_c(eng, name, out, n) bind(C, name='hnumo_get_field')
            import :: c_int, c_ptr, c_char, c_double, c_int64_t
            type(c_ptr), value :: eng
            character(kind=c_char), intent(in) :: name(*)
            real(c_double), intent(out) :: out(*)
            integer(c_int64_t), value :: n
        end function hnumo_get_field_c

        integer(c_int) function hnumo_set_resident(eng, on) bind(C, name='hnumo_set_resident')
            import :: c_int, c_ptr
            type(c_ptr), value :: eng
            integer(c_int), value :: on
        end function hnumo_set_resident

        ! summation order of the barotropic stage: HNUMO_SUM_REFERENCE (default, bitwise) or
        ! HNUMO_SUM_FACTORED (sum-factorised, opt-in; see include/hnumo_engine.h)
        integer(c_int) function hnumo_set_summation(eng, mode) bind(C, name='hnumo_set_summation')
            import :: c_int, c_ptr
            type(c_ptr), value :: eng
            integer(c_int), value :: mode
        end function hnumo_set_summation

        integer(c_int) function hnumo_get_summation(eng) bind(C, name='hnumo_get_summation')
            import :: c_int, c_ptr
            type(c_ptr), value :: eng
        end function hnumo_get_summation

        ! 1: one persistent launch per barotropic sub-cycle, 0: one launch per stage
        integer(c_int) function hnumo_stage_path(eng) bind(C, name='hnumo_stage_path')
            import :: c_int, c_ptr
            type(c_ptr), value :: eng
        end function hnumo_stage_path

        ! residency of the persistent launch, out(8): see hnumo_engine.h
        integer(c_int) function hnumo_persistent_info(eng, out) bind(C, name='hnumo_persistent_info')
            import :: c_int, c_int32_t, c_ptr
            type(c_ptr), value :: eng
            integer(c_int32_t), intent(out) :: out(8)
        end function hnumo_persistent_info

        ! the persistent path over the engine's life, out(4): see hnumo_engine.h (ABI v7)
        integer(c_int) function hnumo_persistent_stats(eng, out) bind(C, name='hnumo_persistent_stats')
            import :: c_int, c_int32_t, c_ptr
            type(c_ptr), value :: eng
            integer(c_int32_t), intent(out) :: out(4)
        end function hnumo_persistent_stats

        ! the prediction half of ti_rk_bcl (ti_rk_bcl.F90:43-57): out q_df2, qb_df, qprime_df2
        integer(c_int) function hnumo_predict(eng, q_df, qb_df, qprime_df) bind(C, name='hnumo_predict')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: eng
            real(c_double), intent(inout) :: q_df(*), qb_df(*), qprime_df(*)
        end function hnumo_predict

        integer(c_int) function hnumo_sync(eng, q_df, qb_df, qprime_df) bind(C, name='hnumo_sync')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: eng
            real(c_double), intent(out) :: q_df(*), qb_df(*), qprime_df(*)
        end function hnumo_sync
    end interface

contains

    ! hnumo_last_error() as a Fortran string
    function hnumo_last_error(eng) result(msg)
        type(c_ptr), intent(in) :: eng
        character(len=:), allocatable :: msg
        character(kind=c_char), pointer :: s(:)
        integer :: n
        call c_f_pointer(hnumo_last_error_c(eng), s, [4096])
        n = 0
        do while (n < 4096)
            if (s(n + 1) == c_null_char) exit
            n = n + 1
        end do
        allocate(character(len=n) :: msg)
        msg = transfer(s(1:n), msg)
    end function hnumo_last_error

    ! copy out a mod_variables equivalent by name, e.g. call hnumo_get_field(eng, 'H_ave', H_ave, rc)
    subroutine hnumo_get_field(eng, name, out, rc)
        type(c_ptr), intent(in) :: eng
        character(len=*), intent(in) :: name
        real(c_double), intent(out) :: out(:)
        integer(c_int), intent(out) :: rc
        rc = hnumo_get_field_c(eng, trim(name) // c_null_char, out, int(size(out), c_int64_t))
    end subroutine hnumo_get_field

end module hnumo_engine_c
