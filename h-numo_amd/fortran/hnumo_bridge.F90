! hnumo_bridge.F90 -- the host side of the drop-in, in h-NUMO's own language.
!
! A module an h-NUMO maintainer adds to src/: it reads the module globals that ti_rk_bcl
! reads (SURVEY.md §8b: mod_grid, mod_face, mod_basis, mod_metrics, mod_initial,
! mod_input, mod_constants, mod_parallel), hands them to libhnumo_engine through the
! ISO_C_BINDING module hnumo_engine_c (include/hnumo_engine.f90), and provides
!
!     call hnumo_bridge_ti_rk_bcl(q_df, qb_df, qprime_df)
!
! with ti_rk_bcl's signature (ti_rk_bcl.F90:9-19), so mod_time_loop.F90:209 changes by one
! name (INTEGRATION.md).  The time averages the reference keeps in mod_variables are copied
! back after each step (hnumo_bridge_fetch_averages) for code that reads them.
!
! Error behaviour mirrors the reference: a negative layer thickness stops the run with the
! reference's message (mod_splitting.F90:74-77); other engine errors stop with the engine's
! message.
module hnumo_bridge

    use iso_c_binding, only: c_int, c_int32_t, c_double, c_ptr, c_null_ptr, c_loc, c_associated, c_char
    use hnumo_engine_c

    implicit none
    private
    public :: hnumo_bridge_init, hnumo_bridge_ti_rk_bcl, hnumo_bridge_fetch_averages, &
        hnumo_bridge_finalize, hnumo_bridge_engine, hnumo_bridge_sync

    type(c_ptr), save :: engine = c_null_ptr

contains

    function hnumo_bridge_engine() result(e)
        type(c_ptr) :: e
        e = engine
    end function hnumo_bridge_engine

    ! address of a contiguous array (descriptors are only read during hnumo_engine_create)
    function pd(a) result(p)
        real(c_double), target, intent(in) :: a(*)
        type(c_ptr) :: p
        p = c_loc(a)
    end function pd

    function pi(a) result(p)
        integer(c_int32_t), target, intent(in) :: a(*)
        type(c_ptr) :: p
        p = c_loc(a)
    end function pi

    ! Build the engine from the module globals after h-NUMO's start-up (mod_initial_mlswe done).
    subroutine hnumo_bridge_init(device, resident)
        use mod_basis, only: ngl, nq, psiq, dpsiq, psi, dpsi
        use mod_grid, only: nelem, npoin, npoin_q, nface, face
        use mod_face, only: imapl, imapr, imapl_q, imapr_q, normal_vector, normal_vector_q, jac_face, jac_faceq
        use mod_metrics, only: massinv, ksiq_x, ksiq_y, etaq_x, etaq_y, jacq, ksi_x, ksi_y, eta_x, eta_y, jac
        use mod_input, only: nlayers, dt, dt_btp, kstages, method_visc, visc_mlswe, botfr, cd_mlswe, ad_mlswe, &
            max_shear_dz
        use mod_constants, only: gravity
        use mod_initial, only: pbprime, pbprime_df, one_over_pbprime, one_over_pbprime_df, pbprime_face, &
            pbprime_df_face, one_over_pbprime_edge, coeff_pbpert_L, coeff_pbpert_R, coeff_pbub_LR, &
            coeff_mass_pbub_L, coeff_mass_pbub_R, coeff_mass_pbpert_LR, alpha_mlswe, tau_wind, &
            coriolis_quad, grad_zbot_quad, zbot_df, zbot_face, fdt2_bcl, a_bcl, b_bcl, ssprk_a, ssprk_beta, N_btp
        use mod_parallel, only: num_nbh, nbh_proc, num_send_recv, nbh_send_recv, nbh_send_recv_multi
        use mod_mpi_utilities, only: irank, numproc
        use mpi
        integer, intent(in) :: device
        logical, intent(in), optional :: resident

        type(hnumo_mesh_desc) :: mesh
        type(hnumo_static_desc) :: st
        type(hnumo_params) :: par
        ! the face arrays carry a dead second face index on this 2-D path: pass (:,:,1,:)
        integer(c_int32_t), allocatable, target :: face8(:, :), imapl1(:, :, :), imapr1(:, :, :)
        integer(c_int32_t), allocatable, target :: imaplq1(:, :, :), imaprq1(:, :, :)
        real(c_double), allocatable, target :: nv1(:, :, :), nvq1(:, :, :), jf1(:, :), jfq1(:, :)
        integer(c_int) :: rc
        ! multi-rank: mod_parallel's processor-face lists as they are, plus an RCCL id from rank 0
        type(hnumo_halo_desc), target :: halo
        integer(c_int32_t), allocatable, target :: h_proc(:), h_num(:), h_list(:)
        character(kind=c_char), allocatable, target :: comm_id(:)
        type(c_ptr) :: halo_p
        integer :: ierr

        if (hnumo_abi_version() /= HNUMO_ABI_EXPECTED) stop 'hnumo_bridge: libhnumo_engine ABI version mismatch'
        halo_p = c_null_ptr
        if (numproc > 1) then
            if (num_nbh > 0) then
                if (any(nbh_send_recv_multi(1:sum(num_send_recv(1:num_nbh))) /= 1)) &
                    stop 'hnumo_bridge: non-conforming processor faces are not supported'
            end if
            allocate(h_proc(max(num_nbh, 1)), h_num(max(num_nbh, 1)), h_list(max(sum(num_send_recv(1:num_nbh)), 1)))
            allocate(comm_id(128))
            h_proc(1:num_nbh) = nbh_proc(1:num_nbh)                ! 1-based ranks, as p4est fills them
            h_num(1:num_nbh) = num_send_recv(1:num_nbh)
            h_list(1:sum(num_send_recv(1:num_nbh))) = nbh_send_recv(1:sum(num_send_recv(1:num_nbh)))
            halo%rank = irank; halo%nranks = numproc; halo%num_nbh = num_nbh
            halo%nbh_proc = c_loc(h_proc); halo%num_send_recv = c_loc(h_num); halo%nbh_send_recv = c_loc(h_list)
            halo%nelem_owned = nelem
            call dump_halo(halo)
            if (irank == 0) then
                rc = hnumo_rccl_unique_id(comm_id)
                if (rc /= HNUMO_OK) stop 'hnumo_bridge: hnumo_rccl_unique_id failed'
            end if
            call mpi_bcast(comm_id, 128, MPI_CHARACTER, 0, MPI_COMM_WORLD, ierr)
            halo%comm_id = c_loc(comm_id)
            halo_p = c_loc(halo)
        end if
        face8 = face(1:8, 1:nface)
        imapl1 = imapl(:, :, 1, :)
        imapr1 = imapr(:, :, 1, :)
        imaplq1 = imapl_q(:, :, 1, :)
        imaprq1 = imapr_q(:, :, 1, :)
        nv1 = normal_vector(:, :, 1, :)
        nvq1 = normal_vector_q(:, :, 1, :)
        jf1 = jac_face(:, 1, :)
        jfq1 = jac_faceq(:, 1, :)

        mesh%nelem = nelem; mesh%npoin = npoin; mesh%npoin_q = npoin_q; mesh%nface = nface
        mesh%ngl = ngl; mesh%nq = nq; mesh%nlayers = nlayers
        mesh%face = c_loc(face8); mesh%imapl = c_loc(imapl1); mesh%imapr = c_loc(imapr1)
        mesh%imapl_q = c_loc(imaplq1); mesh%imapr_q = c_loc(imaprq1)
        mesh%normal_vector = c_loc(nv1); mesh%normal_vector_q = c_loc(nvq1)
        mesh%jac_face = c_loc(jf1); mesh%jac_faceq = c_loc(jfq1)
        mesh%massinv = pd(massinv)
        mesh%psiq = pd(psiq); mesh%dpsiq = pd(dpsiq); mesh%psi = pd(psi); mesh%dpsi = pd(dpsi)
        mesh%ksiq_x = pd(ksiq_x); mesh%ksiq_y = pd(ksiq_y); mesh%etaq_x = pd(etaq_x); mesh%etaq_y = pd(etaq_y)
        mesh%jacq = pd(jacq)
        mesh%ksi_x = pd(ksi_x); mesh%ksi_y = pd(ksi_y); mesh%eta_x = pd(eta_x); mesh%eta_y = pd(eta_y)
        mesh%jac = pd(jac)

        st%pbprime = pd(pbprime); st%pbprime_df = pd(pbprime_df)
        st%one_over_pbprime = pd(one_over_pbprime); st%one_over_pbprime_df = pd(one_over_pbprime_df)
        st%pbprime_face = pd(pbprime_face); st%pbprime_df_face = pd(pbprime_df_face)
        st%one_over_pbprime_edge = pd(one_over_pbprime_edge)
        st%coeff_pbpert_L = pd(coeff_pbpert_L); st%coeff_pbpert_R = pd(coeff_pbpert_R)
        st%coeff_pbub_LR = pd(coeff_pbub_LR); st%coeff_mass_pbub_L = pd(coeff_mass_pbub_L)
        st%coeff_mass_pbub_R = pd(coeff_mass_pbub_R); st%coeff_mass_pbpert_LR = pd(coeff_mass_pbpert_LR)
        st%alpha = pd(alpha_mlswe); st%tau_wind = pd(tau_wind); st%coriolis_quad = pd(coriolis_quad)
        st%grad_zbot_quad = pd(grad_zbot_quad); st%zbot_df = pd(zbot_df); st%zbot_face = pd(zbot_face)
        st%fdt2_bcl = pd(fdt2_bcl); st%a_bcl = pd(a_bcl); st%b_bcl = pd(b_bcl)
        st%ssprk_a = pd(ssprk_a); st%ssprk_beta = pd(ssprk_beta)

        par%dt = dt; par%dt_btp = dt_btp; par%visc_mlswe = visc_mlswe; par%cd_mlswe = cd_mlswe
        par%ad_mlswe = ad_mlswe; par%gravity = gravity; par%max_shear_dz = max_shear_dz
        par%shear_corrector = HNUMO_SHEAR_CORRECTOR_REFERENCE   ! the reference's semantics (hnumo_engine.h)
        par%N_btp = N_btp; par%kstages = kstages; par%method_visc = method_visc; par%botfr = botfr

        rc = hnumo_engine_create(mesh, st, par, halo_p, int(device, c_int), engine)
        if (rc /= HNUMO_OK) then
            print *, 'hnumo_engine_create failed: ', hnumo_last_error(engine)
            stop 'hnumo_bridge_init'
        end if
        if (present(resident)) then
            if (resident) rc = hnumo_set_resident(engine, 1_c_int)
        end if
    end subroutine hnumo_bridge_init

    ! Verification hook (tests/test_fortran_abi.py): with HNUMO_BRIDGE_HALO_DUMP=<path> in the
    ! environment, write the processor-face descriptor exactly as hnumo_engine_create will read it
    ! -- through the descriptor's own pointers -- to <path>.<rank> before the first device call:
    ! int32 rank, nranks, num_nbh, nelem_owned, sum(num_send_recv), then nbh_proc(num_nbh),
    ! num_send_recv(num_nbh), nbh_send_recv(sum).  Nothing is written without the variable.  The
    ! ranks then meet at a barrier, so that rank 0 failing at its first device call cannot end the
    ! job before every rank has written its file.
    subroutine dump_halo(h)
        use iso_c_binding, only: c_f_pointer
        use mpi
        type(hnumo_halo_desc), intent(in) :: h
        character(len=1024) :: path
        character(len=16) :: rs
        integer :: n, stat, u, ierr
        integer(c_int32_t), pointer :: proc(:), num(:), lst(:)
        call get_environment_variable('HNUMO_BRIDGE_HALO_DUMP', path, status=stat)
        if (stat /= 0 .or. len_trim(path) == 0) return
        n = 0
        if (h%num_nbh > 0) then
            call c_f_pointer(h%nbh_proc, proc, [h%num_nbh])
            call c_f_pointer(h%num_send_recv, num, [h%num_nbh])
            n = sum(num)
            call c_f_pointer(h%nbh_send_recv, lst, [max(n, 1)])
        end if
        write(rs, '(I0)') h%rank
        open(newunit=u, file=trim(path) // '.' // trim(rs), access='stream', form='unformatted', status='replace')
        write(u) h%rank, h%nranks, h%num_nbh, h%nelem_owned, int(n, c_int32_t)
        if (h%num_nbh > 0) write(u) proc, num, lst(1:n)
        close(u)
        call mpi_barrier(MPI_COMM_WORLD, ierr)
    end subroutine dump_halo

    ! drop-in for ti_rk_bcl (ti_rk_bcl.F90:9-19): same arguments, same layouts
    subroutine hnumo_bridge_ti_rk_bcl(q_df, qb_df, qprime_df)
        real(c_double), intent(inout) :: q_df(:, :, :), qb_df(:, :), qprime_df(:, :, :)
        integer(c_int) :: rc
        if (.not. c_associated(engine)) stop 'hnumo_bridge_ti_rk_bcl: call hnumo_bridge_init first'
        rc = hnumo_ti_rk_bcl(engine, q_df, qb_df, qprime_df)
        if (rc == HNUMO_ERR_NEGATIVE_THICKNESS) then
            print *, 'Negative mass in thickness at some points'   ! mod_splitting.F90:74-77
            stop
        else if (rc /= HNUMO_OK) then
            print *, 'hnumo_ti_rk_bcl: ', hnumo_last_error(engine)
            stop
        end if
    end subroutine hnumo_bridge_ti_rk_bcl

    ! Resident mode (hnumo_bridge_init(device, resident=.true.)) keeps q_df, qb_df, qprime_df
    ! in HBM between steps and never writes the caller's arrays: call this before anything
    ! on the host reads the state (diagnostics, snapshots, mlswe_FIN.txt, restart dumps --
    ! mod_time_loop.F90:219-254), or those would see the state of the first step.
    subroutine hnumo_bridge_sync(q_df, qb_df, qprime_df)
        real(c_double), intent(inout) :: q_df(:, :, :), qb_df(:, :), qprime_df(:, :, :)
        integer(c_int) :: rc
        if (.not. c_associated(engine)) stop 'hnumo_bridge_sync: call hnumo_bridge_init first'
        rc = hnumo_sync(engine, q_df, qb_df, qprime_df)
        if (rc /= HNUMO_OK) then
            print *, 'hnumo_sync: ', hnumo_last_error(engine)
            stop
        end if
    end subroutine hnumo_bridge_sync

    ! copy the engine's time averages into the reference's mod_variables arrays
    subroutine hnumo_bridge_fetch_averages()
        use mod_variables, only: ope_ave, H_ave, Qu_ave, Qv_ave, Quv_ave, ope2_ave, btp_mass_flux_ave, &
            uvb_ave, tau_bot_ave, tau_wind_ave, ope2_ave_df, uvb_ave_df, uvb_face_ave, &
            btp_mass_flux_face_ave, ope_face_ave, ope2_face_ave, Qu_face_ave, Qv_face_ave, Quv_face_ave, &
            H_face_ave, one_plus_eta_edge_2_ave, graduvb_ave, graduvb_face_ave, Q_uu_dp, Q_uv_dp, Q_vv_dp, &
            H_bcl, Q_uu_dp_edge, Q_uv_dp_edge, Q_vv_dp_edge, H_bcl_edge, btp_dpp_graduv, pbprime_visc, &
            btp_graduv_dpp_face, sum_layer_mass_flux, sum_layer_mass_flux_face, dpprime_visc
        call get('ope_ave', ope_ave); call get('H_ave', H_ave); call get('Qu_ave', Qu_ave)
        call get('Qv_ave', Qv_ave); call get('Quv_ave', Quv_ave); call get('ope2_ave', ope2_ave)
        call get2('btp_mass_flux_ave', btp_mass_flux_ave); call get2('uvb_ave', uvb_ave)
        call get2('tau_bot_ave', tau_bot_ave); call get2('tau_wind_ave', tau_wind_ave)
        call get('ope2_ave_df', ope2_ave_df); call get2('uvb_ave_df', uvb_ave_df)
        call get4('uvb_face_ave', uvb_face_ave); call get3('btp_mass_flux_face_ave', btp_mass_flux_face_ave)
        call get3('ope_face_ave', ope_face_ave); call get3('ope2_face_ave', ope2_face_ave)
        call get3('Qu_face_ave', Qu_face_ave); call get3('Qv_face_ave', Qv_face_ave)
        call get3('Quv_face_ave', Quv_face_ave); call get2('H_face_ave', H_face_ave)
        call get2('one_plus_eta_edge_2_ave', one_plus_eta_edge_2_ave)
        call get2('graduvb_ave', graduvb_ave); call get4('graduvb_face_ave', graduvb_face_ave)
        call get('Q_uu_dp', Q_uu_dp); call get('Q_uv_dp', Q_uv_dp); call get('Q_vv_dp', Q_vv_dp)
        call get('H_bcl', H_bcl); call get2('Q_uu_dp_edge', Q_uu_dp_edge); call get2('Q_uv_dp_edge', Q_uv_dp_edge)
        call get2('Q_vv_dp_edge', Q_vv_dp_edge); call get2('H_bcl_edge', H_bcl_edge)
        call get2('btp_dpp_graduv', btp_dpp_graduv); call get('pbprime_visc', pbprime_visc)
        call get4('btp_graduv_dpp_face', btp_graduv_dpp_face)
        call get2('sum_layer_mass_flux', sum_layer_mass_flux)
        call get3('sum_layer_mass_flux_face', sum_layer_mass_flux_face)
        call get2('dpprime_visc', dpprime_visc)
    contains
        subroutine chk(rc, name)
            integer(c_int), intent(in) :: rc
            character(len=*), intent(in) :: name
            if (rc /= HNUMO_OK) then
                print *, 'hnumo_get_field(', name, '): ', hnumo_last_error(engine)
                stop
            end if
        end subroutine chk
        subroutine get(name, a)
            character(len=*), intent(in) :: name
            real(c_double), intent(inout) :: a(:)
            call chk(hnumo_get_field_c(engine, trim(name) // char(0), a, int(size(a), 8)), name)
        end subroutine get
        subroutine get2(name, a)
            character(len=*), intent(in) :: name
            real(c_double), intent(inout) :: a(:, :)
            call chk(hnumo_get_field_c(engine, trim(name) // char(0), a, int(size(a), 8)), name)
        end subroutine get2
        subroutine get3(name, a)
            character(len=*), intent(in) :: name
            real(c_double), intent(inout) :: a(:, :, :)
            call chk(hnumo_get_field_c(engine, trim(name) // char(0), a, int(size(a), 8)), name)
        end subroutine get3
        subroutine get4(name, a)
            character(len=*), intent(in) :: name
            real(c_double), intent(inout) :: a(:, :, :, :)
            call chk(hnumo_get_field_c(engine, trim(name) // char(0), a, int(size(a), 8)), name)
        end subroutine get4
    end subroutine hnumo_bridge_fetch_averages

    subroutine hnumo_bridge_finalize()
        if (c_associated(engine)) call hnumo_engine_destroy(engine)
        engine = c_null_ptr
    end subroutine hnumo_bridge_finalize

end module hnumo_bridge
