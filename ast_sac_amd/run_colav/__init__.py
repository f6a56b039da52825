"""run_colav (the reference's non-IW two-ship scenario, C1) over the HIP simulator."""
