"""MI355X-native step-5 duplex-consensus path of BSSeqConsensusReads."""
import os as _os

# The host codec's OpenMP teams run on up to five pipeline threads at once (bam.step5_stream:
# decoder, reader, GPU stage, record builder, writer); idle team threads spinning at their barriers
# would take the cores the other stages need (profiles/r03/e2e: 53 -> 37 host CPU seconds per 1M
# families).  libgomp reads this once, when the first library linking it loads (torch may be that
# library), so it is set on package import; a value the user set wins.
_os.environ.setdefault("OMP_WAIT_POLICY", "PASSIVE")
