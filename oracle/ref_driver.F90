! ref_driver.F90 -- TEST INFRASTRUCTURE ONLY (oracle/_ref).
!
! Drives the REFERENCE Fortran hot path (ti_rk_bcl, ti_barotropic_ssprk_mlswe,
! create_rhs_btp and everything below them, compiled unmodified from
! /root/reference/src by oracle/Makefile) on inputs read from a bundle written by
! h-numo_amd/hnumo/bundle.py, and writes its outputs for the parity tests.
!
! The reference's own start-up (p4est mesh, netCDF output, namelists) is not used:
! this program fills the module globals the path reads (SURVEY.md §8b) directly from
! the bundle -- the same arrays the CPU oracle and the HIP engine receive through
! include/hnumo_engine.h.  On one rank (num_nbh = 0) the reference's MPI halo routines run
! with empty neighbour lists; under `mpiexec -n R` every rank reads its own bundle of a
! processor-face partition (<bundle>.<rank>, with mod_parallel's neighbour lists) and the
! reference's own halo exchange (send_receive_bound / create_rhs_communicator) runs over MPI.
!
! usage: ref_driver <bundle.bin> <outputs.bin>
!
! Built a second time with -DHNUMO_DROPIN as oracle/_ref/dropin_driver: the same set-up,
! but mode 3 calls hnumo_bridge_ti_rk_bcl (h-numo_amd/fortran/hnumo_bridge.F90, i.e. the
! HIP engine through the Fortran ISO_C_BINDING module) where the reference calls
! ti_rk_bcl -- the drop-in exactly as INTEGRATION.md describes it.  Its bundle carries the
! per-point metrics (mod_metrics) the bridge reads.
program ref_driver

    use mpi
    use mod_input, only: nopx, nopy, nopz, nlayers, dt, dt_btp, kstages, method_visc, &
        visc_mlswe, botfr, cd_mlswe, ad_mlswe, space_method, is_mlswe, dg_integ_exact, &
        ti_method_btp, is_non_conforming_flg, max_shear_dz
    use mod_basis, only: mod_basis_create, ngl, nq, npts, psiq, dpsiq, psi, dpsi, xgl, wgl, xnq, wnq
    use mod_grid, only: mod_grid_init_unified, npoin, npoin_q, nelem, nface, nboun, face, &
        npoin_cg, nbsido, nNC, face_type
    use mod_face, only: normal_vector, normal_vector_q, jac_face, jac_faceq, imapl, imapr, &
        imapl_q, imapr_q, face_send
    use mod_metrics, only: massinv
#ifdef HNUMO_DROPIN
    use mod_metrics, only: ksiq_x, ksiq_y, etaq_x, etaq_y, jacq, ksi_x, ksi_y, eta_x, eta_y, jac
    use hnumo_bridge, only: hnumo_bridge_init, hnumo_bridge_ti_rk_bcl, hnumo_bridge_fetch_averages, &
        hnumo_bridge_finalize
#endif
    use mod_constants, only: gravity, mod_constants_create
    use mod_initial, only: psih, dpsidx, dpsidy, indexq, wjac, psih_df, dpsidx_df, dpsidy_df, &
        index_df, wjac_df, pbprime, pbprime_df, one_over_pbprime, one_over_pbprime_df, &
        pbprime_face, pbprime_df_face, one_over_pbprime_edge, coeff_pbpert_L, coeff_pbpert_R, &
        coeff_pbub_LR, coeff_mass_pbub_L, coeff_mass_pbub_R, coeff_mass_pbpert_LR, alpha_mlswe, &
        tau_wind, coriolis_quad, coriolis_df, grad_zbot_quad, zbot_df, zbot_face, fdt_bcl, &
        fdt2_bcl, a_bcl, b_bcl, ssprk_a, ssprk_beta, N_btp, nvar
    use mod_variables, only: mod_allocate_mlswe, ope_ave, H_ave, Qu_ave, Qv_ave, Quv_ave, ope2_ave, &
        btp_mass_flux_ave, uvb_ave, tau_bot_ave, tau_wind_ave, ope2_ave_df, uvb_ave_df, &
        uvb_face_ave, btp_mass_flux_face_ave, ope_face_ave, ope2_face_ave, Qu_face_ave, &
        Qv_face_ave, Quv_face_ave, H_face_ave, one_plus_eta_edge_2_ave, graduvb_ave, &
        graduvb_face_ave, Q_uu_dp, Q_uv_dp, Q_vv_dp, H_bcl, Q_uu_dp_edge, Q_uv_dp_edge, &
        Q_vv_dp_edge, H_bcl_edge, btp_dpp_graduv, pbprime_visc, btp_graduv_dpp_face, &
        sum_layer_mass_flux, sum_layer_mass_flux_face, dpprime_visc, dpprime_visc_q
    use mod_mpi_communicator, only: ireq, status
    use mod_parallel, only: num_nbh, num_send_recv, nbh_send_recv, nbh_send_recv_multi, nbh_proc
    use mod_ref, only: q_send, q_recv, recv_data_dg, send_data_dg, lap_q_recv_df1, lap_q_send_df1, &
        lap_recv_data_dg_df1, lap_send_data_dg_df1, recv_data_dg_quad, send_data_dg_quad, nmessage
    use mod_rk_mlswe, only: ti_barotropic_ssprk_mlswe
    use mod_rhs_btp, only: create_rhs_btp
    use mod_barotropic_terms, only: btp_bcl_coeffs_qdf
    use mod_layer_terms, only: extract_qprime_df_face, interpolate_dpp
    use mod_splitting, only: momentum_mass
    use mod_grid, only: coord
    use mod_global_grid, only: npoin_g
    use mod_parallel, only: nproc, npoin_l, npoin_l_max
    use mod_mpi_utilities, only: irank, numproc
    use mod_input, only: lcheck_conserved, test_case, xdims, ydims, f0, beta
    use mod_initial, only: kvector
    use mod_metrics, only: ksiq_x, ksiq_y, etaq_x, etaq_y, jacq
    use mod_initial_mlswe, only: compute_reference_edge_variables, bot_topo_derivatives, &
        wind_stress_coriolis, ssprk_coefficients
    use mod_Tensorproduct, only: compute_gradient_quad
    use mod_basis, only: FACE_LEN

    implicit none

    integer :: hi(16), ierr, u, nsteps, mode, istep, k, ip, I1, myrank, nprocs, nhalo(2)
    character(len=16) :: rsuf
    real(8), allocatable :: qout(:,:,:), mass0(:)
    character(len=18) :: fnp11
    character(len=3) :: s_layers
    real(8) :: t0, t1
    real(8) :: hd(8)
    character(len=512) :: fin, fout
    integer, allocatable :: iface3(:,:,:), iface2(:,:)
    real(8), allocatable :: r3(:,:,:), r2(:,:)
    real(8), allocatable :: q_df(:,:,:), qb_df(:,:), qprime_df(:,:,:), rhs(:,:)
    real(8), allocatable :: qf(:,:,:,:,:)
    integer :: nl, nelem_in, npoin_in, npoin_q_in, nface_in, ngl_in, nq_in, nop_in
    real(8), allocatable :: ref_xgl(:), ref_wgl(:), ref_xnq(:), ref_wnq(:)
    real(8), allocatable :: ref_psiq(:,:), ref_dpsiq(:,:), ref_psi(:,:), ref_dpsi(:,:)
    ! mode 6 (the reference's own set-up routines)
    real(8) :: sp(6)
    real(8), allocatable :: oop_face(:,:,:), pb_edge(:,:), oop_df_face(:,:,:), tw_df(:,:), z_if(:,:), zbot_q(:)
    ! mode 7 (the reference's own metric terms and normals)
    real(8), allocatable :: g_n(:,:,:,:,:), g_q(:,:,:,:,:), g_nv(:,:,:,:), g_jf(:,:,:), g_nvq(:,:,:,:), g_jfq(:,:,:)
    integer, allocatable :: faceL(:,:)

    call mpi_init(ierr)
    call mod_constants_create()                 ! pi, earth_radius (amain.F90:171)
    call mpi_comm_rank(mpi_comm_world, myrank, ierr)
    call mpi_comm_size(mpi_comm_world, nprocs, ierr)
    irank = myrank; numproc = nprocs            ! what initialize_mpi_util sets (mod_mpi_utilities.F90:43-49)
    call get_command_argument(1, fin)
    call get_command_argument(2, fout)
    if (nprocs > 1) then
        ! one bundle per rank (<bundle>.<rank>, a processor-face partition, hnumo/facepart.py)
        write(rsuf, '(I0)') myrank
        fin = trim(fin) // '.' // trim(rsuf)
        fout = trim(fout) // '.' // trim(rsuf)
    end if
    open(newunit=u, file=trim(fin), access='stream', form='unformatted', status='old')
    read(u) hi
    read(u) hd
    nelem_in = hi(1); npoin_in = hi(2); npoin_q_in = hi(3); nface_in = hi(4)
    ngl_in = hi(5); nq_in = hi(6); nl = hi(7); nop_in = hi(8)
    nsteps = hi(13); mode = hi(14)

    ! ---- mod_input (namelist values of the configuration)
    nopx = nop_in; nopy = nop_in; nopz = 0
    nlayers = nl; kstages = hi(9); method_visc = hi(11); botfr = hi(12)
    dt = hd(1); dt_btp = hd(2); visc_mlswe = hd(3); cd_mlswe = hd(4); ad_mlswe = hd(5)
    space_method = 'dg'; is_mlswe = .true.; dg_integ_exact = .true.; ti_method_btp = 'rk35'
    is_non_conforming_flg = 0
    gravity = hd(6); max_shear_dz = hd(7)

    ! ---- mod_basis: the reference builds its own LGL tables (mod_basis.F90:60-186)
    call mod_basis_create(nopx, nopy, nopz)
    if (ngl /= ngl_in .or. nq /= nq_in) stop 'basis size mismatch'

    ! ---- mod_grid (what mod_p4est_create_grid would set, mod_p4est.F90:216-415)
    nelem = nelem_in; nface = nface_in; npoin_cg = npoin_in; nbsido = 0; nNC = 0; nboun = 0
    call mod_grid_init_unified()
    if (npoin /= npoin_in .or. npoin_q /= npoin_q_in) stop 'grid size mismatch'

    allocate(iface2(8, nface)); read(u) iface2; face(1:8, 1:nface) = iface2
    face_type = 0
    allocate(iface3(3, ngl, nface))
    allocate(imapl(3, ngl, ngl, nface), imapr(3, ngl, ngl, nface))
    allocate(imapl_q(3, nq, nq, nface), imapr_q(3, nq, nq, nface))
    imapl = 0; imapr = 0; imapl_q = 0; imapr_q = 0
    read(u) iface3; imapl(:, :, 1, :) = iface3
    read(u) iface3; imapr(:, :, 1, :) = iface3
    deallocate(iface3); allocate(iface3(3, nq, nface))
    read(u) iface3; imapl_q(:, :, 1, :) = iface3
    read(u) iface3; imapr_q(:, :, 1, :) = iface3
    allocate(indexq(npts, npoin_q), index_df(npts, npoin))
    read(u) indexq
    read(u) index_df

    ! ---- mod_face
    allocate(normal_vector(3, ngl, ngl, nface), jac_face(ngl, ngl, nface))
    allocate(normal_vector_q(3, nq, nq, nface), jac_faceq(nq, nq, nface))
    normal_vector = 0; jac_face = 0; normal_vector_q = 0; jac_faceq = 0
    allocate(r3(3, ngl, nface)); read(u) r3; normal_vector(:, :, 1, :) = r3; deallocate(r3)
    allocate(r3(3, nq, nface)); read(u) r3; normal_vector_q(:, :, 1, :) = r3; deallocate(r3)
    allocate(r2(ngl, nface)); read(u) r2; jac_face(:, 1, :) = r2; deallocate(r2)
    allocate(r2(nq, nface)); read(u) r2; jac_faceq(:, 1, :) = r2; deallocate(r2)
    allocate(face_send(0))

    ! ---- mod_metrics
    allocate(massinv(npoin)); read(u) massinv

    ! ---- mod_basis tables: keep the reference's own for the setup check, run with the bundle's
    call write_basis_later()
    allocate(r2(ngl, nq)); read(u) r2; psiq = r2; read(u) r2; dpsiq = r2; deallocate(r2)
    allocate(r2(ngl, ngl)); read(u) r2; psi = r2; read(u) r2; dpsi = r2; deallocate(r2)

    ! ---- mod_initial
    allocate(psih(npts, npoin_q), dpsidx(npts, npoin_q), dpsidy(npts, npoin_q), wjac(npoin_q))
    allocate(psih_df(npts, npoin), dpsidx_df(npts, npoin), dpsidy_df(npts, npoin), wjac_df(npoin))
    psih_df = 0
    read(u) psih; read(u) dpsidx; read(u) dpsidy; read(u) wjac
    read(u) dpsidx_df; read(u) dpsidy_df; read(u) wjac_df
    ! psih_df at the LGL nodes is the identity (read only by compute_conserved)
    do I1 = 1, npoin
        do ip = 1, npts
            if (index_df(ip, I1) == I1) psih_df(ip, I1) = 1
        end do
    end do
    allocate(pbprime(npoin_q), pbprime_df(npoin), one_over_pbprime(npoin_q), one_over_pbprime_df(npoin))
    allocate(pbprime_face(2, nq, nface), pbprime_df_face(2, ngl, nface), one_over_pbprime_edge(nq, nface))
    allocate(coeff_pbpert_L(nq, nface), coeff_pbpert_R(nq, nface), coeff_pbub_LR(nq, nface))
    allocate(coeff_mass_pbub_L(nq, nface), coeff_mass_pbub_R(nq, nface), coeff_mass_pbpert_LR(nq, nface))
    allocate(alpha_mlswe(nlayers), tau_wind(2, npoin_q), coriolis_quad(npoin_q), coriolis_df(npoin))
    allocate(grad_zbot_quad(2, npoin_q), zbot_df(npoin), zbot_face(2, nq, nface))
    allocate(fdt_bcl(npoin), fdt2_bcl(npoin), a_bcl(npoin), b_bcl(npoin))
    allocate(ssprk_a(kstages, 3), ssprk_beta(kstages))
    read(u) pbprime; read(u) pbprime_df; read(u) one_over_pbprime; read(u) one_over_pbprime_df
    read(u) pbprime_face; read(u) pbprime_df_face; read(u) one_over_pbprime_edge
    read(u) coeff_pbpert_L; read(u) coeff_pbpert_R; read(u) coeff_pbub_LR
    read(u) coeff_mass_pbub_L; read(u) coeff_mass_pbub_R; read(u) coeff_mass_pbpert_LR
    read(u) alpha_mlswe; read(u) tau_wind; read(u) coriolis_quad; read(u) grad_zbot_quad
    read(u) zbot_df; read(u) zbot_face; read(u) fdt2_bcl; read(u) a_bcl; read(u) b_bcl
    read(u) ssprk_a; read(u) ssprk_beta
    coriolis_df = 0; fdt_bcl = 2.0d0 * fdt2_bcl
    N_btp = hi(10); nvar = 5

    allocate(q_df(3, npoin, nlayers), qb_df(4, npoin), qprime_df(3, npoin, nlayers), rhs(3, npoin))
    read(u) q_df; read(u) qb_df; read(u) qprime_df
#ifdef HNUMO_DROPIN
    ! ---- mod_metrics per-point metrics (jacq = wjac, jac = wjac_df: Tensor_product.F90:56,91)
    allocate(ksiq_x(nq, nq, 1, nelem), ksiq_y(nq, nq, 1, nelem), etaq_x(nq, nq, 1, nelem))
    allocate(etaq_y(nq, nq, 1, nelem), jacq(nq, nq, 1, nelem))
    allocate(ksi_x(ngl, ngl, 1, nelem), ksi_y(ngl, ngl, 1, nelem), eta_x(ngl, ngl, 1, nelem))
    allocate(eta_y(ngl, ngl, 1, nelem), jac(ngl, ngl, 1, nelem))
    read(u) ksiq_x; read(u) ksiq_y; read(u) etaq_x; read(u) etaq_y; read(u) jacq
    read(u) ksi_x; read(u) ksi_y; read(u) eta_x; read(u) eta_y; read(u) jac
#else
    if (mode == 6) then
        ! mode 6 trailer: quad-point metrics (compute_gradient_quad), node coordinates, and the
        ! namelist values the set-up routines read (xdims, ydims, f0, beta; test_case id hi(16))
        allocate(ksiq_x(nq, nq, 1, nelem), ksiq_y(nq, nq, 1, nelem), etaq_x(nq, nq, 1, nelem))
        allocate(etaq_y(nq, nq, 1, nelem), jacq(nq, nq, 1, nelem))
        read(u) ksiq_x; read(u) ksiq_y; read(u) etaq_x; read(u) etaq_y; read(u) jacq
        read(u) coord
        read(u) sp
        xdims = sp(1:2); ydims = sp(3:4); f0 = sp(5); beta = sp(6)
        select case (hi(16))
        case (1); test_case = 'bump'
        case (2); test_case = 'lakeAtrest'
        case (3); test_case = 'double-gyre'
        case default; stop 'mode 6: unknown test case id'
        end select
    end if
#endif
    if (mode == 7) read(u) coord          ! mode 7 trailer: the DG node coordinates
    if (mode == 5) then
        ! mode 5 trailer: the node coordinates (mod_grid coord, read by courant_mlswe), and the
        ! single-rank gather plumbing of diagnostics / print_diagnostics_mlswe
        read(u) coord
        nproc = 1; irank = 0; npoin_g = npoin; npoin_l_max = npoin
        allocate(npoin_l(1)); npoin_l(1) = npoin
        lcheck_conserved = .true.
    end if
    ! ---- halo plumbing (mod_parallel, mod_mpi_communicator, mod_ref): empty on one rank; the
    ! processor-face lists of p4est (p4est.c:1343-1412) when the bundle carries them
    num_nbh = 0
    nboun = 0
    if (hi(15) == 1) then
        read(u) nhalo
        num_nbh = nhalo(1); nboun = nhalo(2)
        allocate(nbh_proc(num_nbh), num_send_recv(num_nbh), nbh_send_recv(nboun), nbh_send_recv_multi(nboun))
        read(u) nbh_proc; read(u) num_send_recv; read(u) nbh_send_recv
        nbh_send_recv_multi = 1                  ! conforming faces (p4est.c:1707)
        do k = 1, nboun
            face_type(nbh_send_recv(k)) = 2      ! processor face (p4est.c:1691)
        end do
    else
        allocate(num_send_recv(0), nbh_send_recv(0), nbh_send_recv_multi(0), nbh_proc(0))
    end if
    close(u)
    rhs = 0
    allocate(ireq(2 * num_nbh), status(MPI_STATUS_SIZE, 2 * num_nbh))   ! mod_mpi_communicator_create
    ! mod_ref_create's halo buffers (mod_ref.F90:82-118)
    allocate(q_send(4, ngl, nboun), q_recv(4, ngl, nboun), recv_data_dg(4 * ngl * nboun), send_data_dg(4 * ngl * nboun))
    allocate(lap_q_recv_df1(4, ngl, nboun), lap_q_send_df1(4, ngl, nboun))
    allocate(lap_recv_data_dg_df1(4 * ngl * nboun), lap_send_data_dg_df1(4 * ngl * nboun))
    allocate(recv_data_dg_quad(4 * nq * nboun), send_data_dg_quad(4 * nq * nboun))
    nmessage = 6

    ! ---- mod_variables
    call mod_allocate_mlswe()
    call zero_accumulators()
    Q_uu_dp = 0; Q_uv_dp = 0; Q_vv_dp = 0; H_bcl = 0; Q_uu_dp_edge = 0; Q_uv_dp_edge = 0
    Q_vv_dp_edge = 0; H_bcl_edge = 0; btp_dpp_graduv = 0; pbprime_visc = 0; btp_graduv_dpp_face = 0

    ! ---- run the reference path
    select case (mode)
    case (1, 2)
        allocate(qf(3, 2, ngl, nface, nlayers))
        call extract_qprime_df_face(qf, qprime_df)
        dpprime_visc(:, :) = qprime_df(1, :, :)
        if (method_visc == 1) call interpolate_dpp(dpprime_visc_q, dpprime_visc)  ! as ti_rk_bcl.F90:48
        call btp_bcl_coeffs_qdf(qf, qprime_df)
        if (mode == 1) then
            call zero_accumulators()
            call create_rhs_btp(rhs, qb_df, qprime_df)
        else
            call ti_barotropic_ssprk_mlswe(qb_df, qprime_df)
        end if
    case (3)
#ifdef HNUMO_DROPIN
        call hnumo_bridge_init(0)
        t0 = mpi_wtime()
        do istep = 1, nsteps
            call hnumo_bridge_ti_rk_bcl(q_df, qb_df, qprime_df)
        end do
        t1 = mpi_wtime()
        call hnumo_bridge_fetch_averages()
        call hnumo_bridge_finalize()
        write(*, '(A,ES24.16)') 'DROPIN_TIME ', t1 - t0
#else
        t0 = mpi_wtime()
        do istep = 1, nsteps
            call ti_rk_bcl(q_df, qb_df, qprime_df)
        end do
        t1 = mpi_wtime()
        write(*, '(A,ES24.16)') 'REF_TIME ', t1 - t0
#endif
    case (4)
        ! the prediction half of ti_rk_bcl (ti_rk_bcl.F90:43-57), outputs q_df2, qbp_df,
        ! qprime_df2: pins momentum_mass (with ad_mlswe > 0, the vertical shear stress)
        allocate(qf(3, 2, ngl, nface, nlayers))
        call extract_qprime_df_face(qf, qprime_df)
        dpprime_visc(:, :) = qprime_df(1, :, :)
        if (method_visc == 1) call interpolate_dpp(dpprime_visc_q, dpprime_visc)
        call btp_bcl_coeffs_qdf(qf, qprime_df)
        call ti_barotropic_ssprk_mlswe(qb_df, qprime_df)
        call momentum_mass(q_df, qf, qprime_df, qb_df)
    case (5)
        ! the diagnostics of the time loop (mod_time_loop.F90:150-186, :257-268): initial layer
        ! masses, nsteps of ti_rk_bcl, then print_diagnostics_mlswe with idone = 0 (stdout
        ! report + mass_mlswe.cons line) and idone = 1 (final report + mlswe_FIN.txt)
        allocate(qout(5, npoin, nlayers), mass0(nlayers))
        call diagnostics(qout, q_df, qb_df, 0, 1)
        do k = 1, nlayers
            call compute_conserved(mass0(k), qout(1, :, k))
        end do
        do istep = 1, nsteps
            call ti_rk_bcl(q_df, qb_df, qprime_df)
        end do
        call diagnostics(qout, q_df, qb_df, nsteps, 1)
        write(s_layers, '(i3)') nlayers
        fnp11 = '(i8,' // trim(adjustl(s_layers)) // '(e16.8,1x))'
        open(unit=111, file='mass_mlswe.cons')
        call print_diagnostics_mlswe(qout, qb_df, dt*nsteps, nsteps, dt, 0, mass0, nsteps, fnp11, 111)
        close(111)
        call print_diagnostics_mlswe(qout, qb_df, dt*nsteps, nsteps, dt, 1, mass0, nsteps, fnp11, 111)
    case (6)
        ! The reference's own start-up of the MLSWE fields, in mod_initial_create's order
        ! (mod_initial.F90:159-183) on the harness mesh: initial_conditions (ICs, pbprime at
        ! nodes / quad points / faces and the reciprocals), compute_reference_edge_variables
        ! (the wave-speed edge coefficients), bot_topo_derivatives (zbot, zbot_face),
        ! compute_gradient_quad (grad_zbot_quad), N_btp, wind_stress_coriolis (wind, Coriolis,
        ! implicit-Coriolis coefficients), ssprk_coefficients.  Pins hnumo/case.py (a18).
        allocate(kvector(3, npoin))
        allocate(oop_face(2, nq, nface), pb_edge(nq, nface), oop_df_face(2, ngl, nface))
        allocate(tw_df(2, npoin), z_if(npoin, nlayers + 1), zbot_q(npoin_q))
        ! initial_conditions accumulates into its never-zeroed automatic array
        ! one_plus_eta_temp (initial_conditions.F90:43,382), which the reference build's
        ! -finit-real=zero starts at 0 (SURVEY Appendix B.12): zero the stack it will occupy
        call zero_stack(64 * (npoin + npoin_q) * (nlayers + 2))
        call initial_conditions(q_df, pbprime, pbprime_df, pbprime_face, one_over_pbprime, oop_face, pb_edge, &
            one_over_pbprime_edge, one_over_pbprime_df, qb_df, qprime_df, alpha_mlswe, oop_df_face, &
            pbprime_df_face, zbot_df, tw_df, z_if)
        call compute_reference_edge_variables(coeff_pbpert_L, coeff_pbpert_R, coeff_pbub_LR, &
            coeff_mass_pbub_L, coeff_mass_pbub_R, coeff_mass_pbpert_LR, pbprime_face, alpha_mlswe)
        zbot_q = 0   ! bot_topo_derivatives accumulates into zbot unzeroed (SURVEY Appendix B.12)
        call bot_topo_derivatives(zbot_q, zbot_face, zbot_df)
        call compute_gradient_quad(grad_zbot_quad, zbot_df)
        N_btp = ceiling(dt / dt_btp)
        dt_btp = dt / real(N_btp)
        call wind_stress_coriolis(tau_wind, coriolis_df, coriolis_quad, fdt_bcl, fdt2_bcl, a_bcl, b_bcl, tw_df)
        call ssprk_coefficients(ssprk_a, ssprk_beta)
        open(newunit=u, file=trim(fout), access='stream', form='unformatted', status='replace')
        write(u) q_df, qb_df, qprime_df, pbprime, pbprime_df, pbprime_face, pbprime_df_face
        write(u) one_over_pbprime, one_over_pbprime_df, one_over_pbprime_edge
        write(u) coeff_pbpert_L, coeff_pbpert_R, coeff_pbub_LR, coeff_mass_pbub_L, coeff_mass_pbub_R
        write(u) coeff_mass_pbpert_LR, alpha_mlswe, zbot_df, zbot_face, grad_zbot_quad, tau_wind
        write(u) coriolis_quad, fdt2_bcl, a_bcl, b_bcl, ssprk_a, ssprk_beta, real(N_btp, 8), dt_btp, gravity
        close(u)
        call mpi_finalize(ierr)
        stop
    case (7)
        ! The reference's geometry of the harness mesh (what mod_metrics_create / mod_face_create
        ! compute at start-up from p4est's node coordinates): metrics (metrics.F90), metrics_quad
        ! (metrics_quad.F90), create_normals (create_normals.F90), create_normals_quad
        ! (create_normals_quad.F90), on the bundle's coordinates (intma = intma_dg) and faces.
        ! Pins hnumo/quadmesh.py (row f3, general quadrilateral grids).
        allocate(g_n(ngl, ngl, 1, nelem, 11), g_q(nq, nq, 1, nelem, 11))
        allocate(g_nv(3, ngl, ngl, nface), g_jf(ngl, ngl, nface), g_nvq(3, nq, nq, nface), g_jfq(nq, nq, nface))
        allocate(faceL(FACE_LEN, nface)); faceL = 0; faceL(1:8, :) = face(1:8, 1:nface)
        call metrics(g_n(:,:,:,:,1), g_n(:,:,:,:,2), g_n(:,:,:,:,3), g_n(:,:,:,:,4), g_n(:,:,:,:,5), &
            g_n(:,:,:,:,6), g_n(:,:,:,:,7), g_n(:,:,:,:,8), g_n(:,:,:,:,9), g_n(:,:,:,:,10), g_n(:,:,:,:,11))
        call metrics_quad(g_q(:,:,:,:,1), g_q(:,:,:,:,2), g_q(:,:,:,:,3), g_q(:,:,:,:,4), g_q(:,:,:,:,5), &
            g_q(:,:,:,:,6), g_q(:,:,:,:,7), g_q(:,:,:,:,8), g_q(:,:,:,:,9), g_q(:,:,:,:,10), g_q(:,:,:,:,11))
        call create_normals(g_nv, g_jf, faceL, nface)
        call create_normals_quad(g_nvq, g_jfq, faceL, nface)
        open(newunit=u, file=trim(fout), access='stream', form='unformatted', status='replace')
        ! ksi_x, ksi_y, eta_x, eta_y, jac at the nodes and at the quadrature points
        write(u) g_n(:,:,1,:,1), g_n(:,:,1,:,2), g_n(:,:,1,:,4), g_n(:,:,1,:,5), g_n(:,:,1,:,10)
        write(u) g_q(:,:,1,:,1), g_q(:,:,1,:,2), g_q(:,:,1,:,4), g_q(:,:,1,:,5), g_q(:,:,1,:,10)
        write(u) g_nv(:,:,1,:), g_jf(:,1,:), g_nvq(:,:,1,:), g_jfq(:,1,:)
        close(u)
        call mpi_finalize(ierr)
        stop
    case default
        stop 'unknown mode'
    end select

    ! ---- outputs
    open(newunit=u, file=trim(fout), access='stream', form='unformatted', status='replace')
    write(u) q_df, qb_df, qprime_df, rhs
    write(u) ope_ave, H_ave, Qu_ave, Qv_ave, Quv_ave, ope2_ave, btp_mass_flux_ave, uvb_ave
    write(u) tau_bot_ave, tau_wind_ave, ope2_ave_df, uvb_ave_df, uvb_face_ave
    write(u) btp_mass_flux_face_ave, ope_face_ave, ope2_face_ave, Qu_face_ave, Qv_face_ave
    write(u) Quv_face_ave, H_face_ave, one_plus_eta_edge_2_ave, graduvb_ave, graduvb_face_ave
    write(u) Q_uu_dp, Q_uv_dp, Q_vv_dp, H_bcl, Q_uu_dp_edge, Q_uv_dp_edge, Q_vv_dp_edge, H_bcl_edge
    write(u) btp_dpp_graduv, pbprime_visc, btp_graduv_dpp_face, sum_layer_mass_flux
    write(u) sum_layer_mass_flux_face
    write(u) ref_xgl, ref_wgl, ref_xnq, ref_wnq, ref_psiq, ref_dpsiq, ref_psi, ref_dpsi
    close(u)
    call mpi_finalize(ierr)

contains

    subroutine write_basis_later()
        allocate(ref_xgl(ngl), ref_wgl(ngl), ref_xnq(nq), ref_wnq(nq))
        allocate(ref_psiq(ngl, nq), ref_dpsiq(ngl, nq), ref_psi(ngl, ngl), ref_dpsi(ngl, ngl))
        ref_xgl = xgl; ref_wgl = wgl; ref_xnq = xnq; ref_wnq = wnq
        ref_psiq = psiq; ref_dpsiq = dpsiq; ref_psi = psi; ref_dpsi = dpsi
    end subroutine write_basis_later

    ! a zero-filled stack region below the caller's frame, for the next call's uninitialised
    ! automatic arrays (volatile: the stores are not optimised away)
    subroutine zero_stack(n)
        integer, intent(in) :: n
        real(8), volatile :: buf(n)
        buf = 0
    end subroutine zero_stack

    ! accumulators are zeroed by ti_barotropic_ssprk_mlswe (mod_rk_mlswe.F90:45-72); a lone
    ! create_rhs_btp call (mode 1) needs the same starting point.
    subroutine zero_accumulators()
        ope_ave = 0; H_ave = 0; Qu_ave = 0; Qv_ave = 0; Quv_ave = 0; ope2_ave = 0
        btp_mass_flux_ave = 0; uvb_ave = 0; tau_bot_ave = 0; tau_wind_ave = 0
        ope2_ave_df = 0; uvb_ave_df = 0; uvb_face_ave = 0; btp_mass_flux_face_ave = 0
        ope_face_ave = 0; ope2_face_ave = 0; Qu_face_ave = 0; Qv_face_ave = 0
        Quv_face_ave = 0; H_face_ave = 0; one_plus_eta_edge_2_ave = 0; graduvb_ave = 0
        graduvb_face_ave = 0; sum_layer_mass_flux = 0; sum_layer_mass_flux_face = 0
    end subroutine zero_accumulators

end program ref_driver
