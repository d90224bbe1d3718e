"""MI355X-native temporal inverse kinematics (ST-GCN IK + SMPL-X FK) engine."""
