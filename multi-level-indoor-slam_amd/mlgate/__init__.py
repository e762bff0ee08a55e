"""mlgate -- MI355X-native semantic loop-closure gate.

Drop-in for the hot path of wadewilliamsw1234/Multi-level-Indoor-SLAM's
``scripts.semantic_gating`` package (VPR descriptors, all-keyframes cosine kNN, floor
gate, geometric verification): the same public names, signatures and return types,
computed by hand-written gfx950 HIP kernels behind the C ABI in include/mlgate.h.

    from mlgate import SemanticPlaceRecognition, SemanticLoopClosureGate   # was
    from scripts.semantic_gating import SemanticPlaceRecognition, ...       # reference

Out of scope (not on the gate's hot path): SemanticGatingPipeline and
the three trajectory-analysis integrations' file loading / plotting (their candidate
generator + gate is mlgate.proximity.TrajectoryLoopClosureGate).
"""
from .floors import ElevatorEvent, IMUFloorDetector, load_imu_from_bag
from .gate import ContextualPriorFactor, LoopClosureCandidate, SemanticLoopClosureGate, integrate_with_orbslam3
from .lidar import FloorEstimate, LiDARFloorTracker, MultiModalFloorDetector
from .verify import (GeometricVerifier, LightGlue, LoFTR, MatchResult, SemanticGeometricVerifier, SuperGlue)
from .vpr import (AnyLoc, CricaVPR, MixVPR, PlaceDescriptor, PlaceMatch, SALAD, SemanticPlaceRecognition,
                  process_image_sequence)

__all__ = [
    'IMUFloorDetector', 'ElevatorEvent', 'load_imu_from_bag',
    'LiDARFloorTracker', 'MultiModalFloorDetector', 'FloorEstimate',
    'SemanticLoopClosureGate', 'LoopClosureCandidate', 'ContextualPriorFactor', 'integrate_with_orbslam3',
    'MixVPR', 'SALAD', 'AnyLoc', 'CricaVPR', 'SemanticPlaceRecognition', 'PlaceMatch', 'PlaceDescriptor',
    'process_image_sequence',
    'LightGlue', 'SuperGlue', 'LoFTR', 'GeometricVerifier', 'SemanticGeometricVerifier', 'MatchResult',
]

__version__ = '0.1.0'
