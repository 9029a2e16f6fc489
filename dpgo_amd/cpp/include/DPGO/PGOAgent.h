// PGOAgent, RBCD-round portion (reference include/DPGO/PGOAgent.h:59-726, src/PGOAgent.cpp).
// The per-round arithmetic (updateX -> QuadraticOptimizer) runs on the GPU; Q/G assembly, GNC
// weights, Nesterov bookkeeping and the robust global-frame initialisation (:250-432) stay on the
// host, as in the reference.  Out of scope: async optimisation thread, logging.
#ifndef DPGO_AMD_PGOAGENT_H
#define DPGO_AMD_PGOAGENT_H

#include <DPGO/DPGO_robust.h>
#include <DPGO/DPGO_types.h>
#include <DPGO/QuadraticProblem.h>
#include <DPGO/RelativeSEMeasurement.h>

#include <memory>
#include <optional>
#include <set>
#include <string>
#include <vector>

namespace DPGO {

enum PGOAgentState { WAIT_FOR_DATA, WAIT_FOR_INITIALIZATION, INITIALIZED };

struct PGOAgentParameters {
  unsigned d, r, numRobots;
  ROPTALG algorithm;
  bool multirobot_initialization;
  bool acceleration;
  unsigned restartInterval;
  RobustCostType robustCostType;
  RobustCostParameters robustCostParams;
  bool robustOptWarmStart;
  unsigned robustOptInnerIters;
  double robustOptMinConvergenceRatio;
  unsigned maxNumIters;
  double relChangeTol;
  bool verbose, logData;
  std::string logDirectory;
  PGOAgentParameters(unsigned dIn, unsigned rIn, unsigned numRobotsIn = 1, ROPTALG algorithmIn = ROPTALG::RTR,
                     bool accel = false, unsigned restartInt = 30, RobustCostType costType = RobustCostType::GNC_TLS,
                     RobustCostParameters costParams = RobustCostParameters(), bool robust_opt_warm_start = true,
                     unsigned robust_opt_inner_iters = 30, double robust_opt_min_convergence_ratio = 0.8,
                     unsigned maxIters = 500, double changeTol = 5e-3, bool v = false, bool log = false,
                     std::string logDir = "")
      : d(dIn), r(rIn), numRobots(numRobotsIn), algorithm(algorithmIn), multirobot_initialization(true),
        acceleration(accel), restartInterval(restartInt), robustCostType(costType), robustCostParams(costParams),
        robustOptWarmStart(robust_opt_warm_start), robustOptInnerIters(robust_opt_inner_iters),
        robustOptMinConvergenceRatio(robust_opt_min_convergence_ratio), maxNumIters(maxIters),
        relChangeTol(changeTol), verbose(v), logData(log), logDirectory(std::move(logDir)) {}
};

struct PGOAgentStatus {
  unsigned agentID;
  PGOAgentState state;
  unsigned instanceNumber, iterationNumber;
  bool readyToTerminate;
  double relativeChange;
  explicit PGOAgentStatus(unsigned id, PGOAgentState s = WAIT_FOR_DATA, unsigned instance = 0,
                          unsigned iteration = 0, bool ready = false, double rel = 0)
      : agentID(id), state(s), instanceNumber(instance), iterationNumber(iteration), readyToTerminate(ready),
        relativeChange(rel) {}
};

class PGOAgent {
 public:
  PGOAgent(unsigned ID, const PGOAgentParameters& params);
  ~PGOAgent();

  void setPoseGraph(const std::vector<RelativeSEMeasurement>& inputOdometry,
                    const std::vector<RelativeSEMeasurement>& inputPrivateLoopClosures,
                    const std::vector<RelativeSEMeasurement>& inputSharedLoopClosures,
                    const Matrix& TInit = Matrix());
  void setX(const Matrix& Xin);
  bool getX(Matrix& Mout);
  bool getSharedPose(unsigned index, Matrix& Mout);
  bool getAuxSharedPose(unsigned index, Matrix& Mout);
  bool getSharedPoseDict(PoseDict& map);
  bool getAuxSharedPoseDict(PoseDict& map);
  void setLiftingMatrix(const Matrix& M);
  bool getLiftingMatrix(Matrix& M) const;
  void updateNeighborPoses(unsigned neighborID, const PoseDict& poseDict);
  void updateAuxNeighborPoses(unsigned neighborID, const PoseDict& poseDict);
  void iterate(bool doOptimization = true);
  bool getTrajectoryInLocalFrame(Matrix& Trajectory);
  Matrix localPoseGraphOptimization();
  void setGlobalAnchor(const Matrix& M) { globalAnchor = M; }
  // robust global-frame initialisation (reference include/DPGO/PGOAgent.h:449-474)
  Matrix computeNeighborTransform(const PoseID& nID, const Matrix& var);
  Matrix computeRobustNeighborTransformTwoStage(unsigned neighborID, const PoseDict& poseDict);
  Matrix computeRobustNeighborTransform(unsigned neighborID, const PoseDict& poseDict);
  void initializeInGlobalFrame(unsigned neighborID, const PoseDict& poseDict);

  unsigned getID() const { return mID; }
  unsigned num_poses() const { return n; }
  unsigned dimension() const { return d; }
  unsigned relaxation_rank() const { return r; }
  unsigned instance_number() const { return 0; }
  unsigned iteration_number() const { return mIterationNumber; }
  PGOAgentState getState() const { return mState; }
  PGOAgentStatus getStatus() {  // reference include/DPGO/PGOAgent.h:285-291
    mStatus.agentID = mID;
    mStatus.state = mState;
    mStatus.iterationNumber = mIterationNumber;
    return mStatus;
  }
  void setNeighborStatus(const PGOAgentStatus& s);
  PGOAgentStatus getNeighborStatus(unsigned id) const;
  std::vector<unsigned> getNeighbors() const { return std::vector<unsigned>(neighborRobotIDs.begin(), neighborRobotIDs.end()); }
  const ROPTResult& lastOptResult() const { return mLastResult; }

 private:
  void addOdometry(const RelativeSEMeasurement& m);
  void addPrivateLoopClosure(const RelativeSEMeasurement& m);
  void addSharedLoopClosure(const RelativeSEMeasurement& m);
  RelativeSEMeasurement& findSharedLoopClosureWithNeighbor(const PoseID& nID);
  void collectNeighborTransforms(const PoseDict& poseDict, std::vector<Matrix>& RVec, std::vector<Vector>& tVec);
  void constructQMatrix();
  bool constructGMatrix(const PoseDict& poseDict);
  bool updateX(bool doOptimization, bool acceleration);
  void initializeAcceleration();
  void updateGamma();
  void updateAlpha();
  void updateY();
  void updateV();
  bool shouldRestart() const;
  void restartNesterovAcceleration(bool doOptimization);
  bool shouldUpdateLoopClosureWeights() const;
  void updateLoopClosuresWeights();
  double computeConvergedLoopClosureRatio() const;

  unsigned mID, d, r, n;
  PGOAgentParameters mParams;
  PGOAgentState mState;
  PGOAgentStatus mStatus;
  RobustCost mRobustCost;
  std::unique_ptr<QuadraticProblem> mProblem;
  unsigned mIterationNumber = 0;
  std::vector<RelativeSEMeasurement> odometry, privateLoopClosures, sharedLoopClosures;
  std::set<PoseID> localSharedPoseIDs, neighborSharedPoseIDs;
  std::set<unsigned> neighborRobotIDs;
  std::vector<PGOAgentStatus> mTeamStatus;
  PoseDict neighborPoseDict, neighborAuxPoseDict;
  Matrix X, XPrev, Y, V;
  std::optional<Matrix> XInit, YLift, TLocalInit, globalAnchor;
  double gamma = 0, alpha = 0;
  ROPTResult mLastResult;
};

}  // namespace DPGO

#endif
