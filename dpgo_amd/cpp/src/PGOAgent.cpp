// PGOAgent RBCD-round portion (reference src/PGOAgent.cpp); see PGOAgent.h.
#include <DPGO/DPGO_utils.h>
#include <DPGO/PGOAgent.h>
#include <DPGO/QuadraticOptimizer.h>
#include <DPGO/manifold/LiftedSEManifold.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <stdexcept>

namespace DPGO {

// ---------------------------------------------------------------- RobustCost (src/DPGO_robust.cpp)
RobustCost::RobustCost(RobustCostType type, const RobustCostParameters& params) : mCostType(type), mParams(params) {
  reset();
}

double RobustCost::weight(double rr) const {
  switch (mCostType) {
    case L2: return 1;
    case L1: return 1 / rr;
    case Huber: return rr < mParams.HuberThreshold ? 1 : mParams.HuberThreshold / rr;
    case TLS: return rr < mParams.TLSThreshold ? 1 : 0;
    case GM: {
      const double a = 1 + rr * rr;
      return 1 / (a * a);
    }
    case GNC_TLS: {  // eq. (14) of the GNC paper (:48-61)
      const double rSq = rr * rr, bc = mParams.GNCBarc * mParams.GNCBarc;
      if (rSq >= (mu + 1) / mu * bc) return 0;
      if (rSq <= mu / (mu + 1) * bc) return 1;
      return std::sqrt(bc * mu * (mu + 1) / rSq) - mu;
    }
  }
  throw std::runtime_error("weight function for selected cost function is not implemented");
}

void RobustCost::reset() {
  mu = mParams.GNCInitMu;
  mGNCIteration = 0;
}

double RobustCost::computeErrorThresholdAtQuantile(double quantile, size_t dimension) {
  if (dimension != 3 || !(quantile > 0)) throw std::invalid_argument("computeErrorThresholdAtQuantile: 3D only");
  return quantile < 1 ? std::sqrt(chi2inv(quantile, 6)) : 1e5;
}

void RobustCost::update() {
  if (mCostType != GNC_TLS) return;
  if (++mGNCIteration > mParams.GNCMaxNumIters) return;
  mu = mParams.GNCMuStep * mu;
}

// ---------------------------------------------------------------- PGOAgent
PGOAgent::PGOAgent(unsigned ID, const PGOAgentParameters& params)
    : mID(ID), d(params.d), r(params.r), n(1), mParams(params), mState(WAIT_FOR_DATA), mStatus(ID),
      mRobustCost(params.robustCostType, params.robustCostParams) {
  X = Matrix::Zero(r, d + 1);
  X.setBlock(0, 0, Matrix::Identity(d, d));
  if (mID == 0) setLiftingMatrix(fixedStiefelVariable(d, r));  // :48
  for (unsigned i = 0; i < mParams.numRobots; ++i) mTeamStatus.emplace_back(i);
}

PGOAgent::~PGOAgent() = default;

void PGOAgent::setLiftingMatrix(const Matrix& M) {
  if (M.rows() != r || M.cols() != d) throw std::invalid_argument("lifting matrix must be r x d");
  YLift = M;
}

bool PGOAgent::getLiftingMatrix(Matrix& M) const {
  if (!YLift) return false;
  M = *YLift;
  return true;
}

void PGOAgent::addOdometry(const RelativeSEMeasurement& m) {
  n = std::max<unsigned>(n, static_cast<unsigned>(m.p2) + 1);
  odometry.push_back(m);
}

void PGOAgent::addPrivateLoopClosure(const RelativeSEMeasurement& m) {
  n = std::max<unsigned>(n, static_cast<unsigned>(std::max(m.p1, m.p2)) + 1);
  privateLoopClosures.push_back(m);
}

void PGOAgent::addSharedLoopClosure(const RelativeSEMeasurement& m) {  // :223-248
  if (m.r1 == mID) {
    n = std::max<unsigned>(n, static_cast<unsigned>(m.p1) + 1);
    localSharedPoseIDs.insert({mID, static_cast<unsigned>(m.p1)});
    neighborSharedPoseIDs.insert({static_cast<unsigned>(m.r2), static_cast<unsigned>(m.p2)});
    neighborRobotIDs.insert(static_cast<unsigned>(m.r2));
  } else {
    n = std::max<unsigned>(n, static_cast<unsigned>(m.p2) + 1);
    localSharedPoseIDs.insert({mID, static_cast<unsigned>(m.p2)});
    neighborSharedPoseIDs.insert({static_cast<unsigned>(m.r1), static_cast<unsigned>(m.p1)});
    neighborRobotIDs.insert(static_cast<unsigned>(m.r1));
  }
  sharedLoopClosures.push_back(m);
}

void PGOAgent::setPoseGraph(const std::vector<RelativeSEMeasurement>& inputOdometry,
                            const std::vector<RelativeSEMeasurement>& inputPrivateLoopClosures,
                            const std::vector<RelativeSEMeasurement>& inputSharedLoopClosures, const Matrix& TInit) {
  if (mState != WAIT_FOR_DATA) throw std::logic_error("setPoseGraph: pose graph already set");
  if (inputOdometry.empty()) return;
  for (const auto& e : inputOdometry) addOdometry(e);
  for (const auto& e : inputPrivateLoopClosures) addPrivateLoopClosure(e);
  for (const auto& e : inputSharedLoopClosures) addSharedLoopClosure(e);
  mProblem.reset(new QuadraticProblem(n, d, r));
  constructQMatrix();
  if (TInit.rows() == d && TInit.cols() == static_cast<long>((d + 1) * n)) {
    TLocalInit = TInit;
  } else {
    // localInitialization (:947-962): chordal for the L2 cost; with a robust cost the loop closures
    // are not trusted and the odometry chain is used
    if (mParams.robustCostType == RobustCostType::L2) {
      std::vector<RelativeSEMeasurement> ms = odometry;
      ms.insert(ms.end(), privateLoopClosures.begin(), privateLoopClosures.end());
      TLocalInit = chordalInitialization(d, n, ms);
    } else {
      TLocalInit = odometryInitialization(d, n, odometry);
    }
  }
  mState = WAIT_FOR_INITIALIZATION;
  if (mID == 0 || !mParams.multirobot_initialization) {
    if (!YLift) throw std::logic_error("setPoseGraph: lifting matrix not set");
    X = (*YLift) * (*TLocalInit);
    XInit = X;
    mState = INITIALIZED;
    if (mParams.acceleration) initializeAcceleration();
  }
}

void PGOAgent::setX(const Matrix& Xin) {  // :55-68
  if (mState == WAIT_FOR_DATA) throw std::logic_error("setX before setPoseGraph");
  if (Xin.rows() != r || Xin.cols() != static_cast<long>((d + 1) * n)) throw std::invalid_argument("setX: bad size");
  mState = INITIALIZED;
  X = Xin;
  if (!XInit) XInit = X;
  if (mParams.acceleration) initializeAcceleration();
}

bool PGOAgent::getX(Matrix& Mout) {
  Mout = X;
  return true;
}

bool PGOAgent::getSharedPose(unsigned index, Matrix& Mout) {
  if (mState != INITIALIZED || index >= n) return false;
  Mout = X.block(0, index * (d + 1), r, d + 1);
  return true;
}

bool PGOAgent::getAuxSharedPose(unsigned index, Matrix& Mout) {
  if (mState != INITIALIZED || index >= n || !mParams.acceleration) return false;
  Mout = Y.block(0, index * (d + 1), r, d + 1);
  return true;
}

bool PGOAgent::getSharedPoseDict(PoseDict& map) {  // :95-106
  if (mState != INITIALIZED) return false;
  map.clear();
  for (const auto& id : localSharedPoseIDs) map[id] = X.block(0, id.second * (d + 1), r, d + 1);
  return true;
}

bool PGOAgent::getAuxSharedPoseDict(PoseDict& map) {  // :108-118
  if (mState != INITIALIZED || !mParams.acceleration) return false;
  map.clear();
  for (const auto& id : localSharedPoseIDs) map[id] = Y.block(0, id.second * (d + 1), r, d + 1);
  return true;
}

void PGOAgent::setNeighborStatus(const PGOAgentStatus& s) {
  if (s.agentID < mTeamStatus.size()) mTeamStatus[s.agentID] = s;
}

PGOAgentStatus PGOAgent::getNeighborStatus(unsigned id) const { return mTeamStatus.at(id); }

// ---------------------------------------------------------------- global-frame initialisation
RelativeSEMeasurement& PGOAgent::findSharedLoopClosureWithNeighbor(const PoseID& nID) {  // :922-934
  for (auto& m : sharedLoopClosures)
    if ((m.r1 == nID.first && m.p1 == nID.second) || (m.r2 == nID.first && m.p2 == nID.second)) return m;
  throw std::runtime_error("Cannot find shared loop closure with neighbor.");
}

Matrix PGOAgent::computeNeighborTransform(const PoseID& nID, const Matrix& var) {  // :250-287
  if (!YLift || !TLocalInit) throw std::logic_error("computeNeighborTransform: lifting matrix / local init missing");
  const RelativeSEMeasurement& m = findSharedLoopClosureWithNeighbor(nID);
  const long b = d + 1;
  Matrix dT = Matrix::Identity(b, b);
  dT.setBlock(0, 0, m.R);
  dT.setBlock(0, d, m.t);
  // the neighbour's pose rounded back to SE(d) in its (already global) frame
  Matrix Tw2f2 = Matrix::Identity(b, b);
  Tw2f2.setBlock(0, 0, YLift->transpose() * var);
  Matrix Tf1f2, Tw1f1 = Matrix::Identity(b, b);
  if (m.r1 == nID.first) {  // incoming edge: neighbour -> me
    Tf1f2 = dT.inverse();
    Tw1f1.setBlock(0, 0, TLocalInit->block(0, m.p2 * b, d, b));
  } else {  // outgoing edge: me -> neighbour
    Tf1f2 = dT;
    Tw1f1.setBlock(0, 0, TLocalInit->block(0, m.p1 * b, d, b));
  }
  const Matrix Tw2w1 = Tw2f2 * Tf1f2.inverse() * Tw1f1.inverse();
  checkRotationMatrix(Tw2w1.block(0, 0, d, d));
  return Tw2w1;
}

void PGOAgent::collectNeighborTransforms(const PoseDict& poseDict, std::vector<Matrix>& RVec,
                                         std::vector<Vector>& tVec) {
  for (const auto& kv : poseDict) {
    if (neighborSharedPoseIDs.find(kv.first) == neighborSharedPoseIDs.end()) continue;
    const Matrix T = computeNeighborTransform(kv.first, kv.second);
    RVec.push_back(T.block(0, 0, d, d));
    tVec.push_back(T.block(0, d, d, 1));
  }
}

Matrix PGOAgent::computeRobustNeighborTransformTwoStage(unsigned neighborID, const PoseDict& poseDict) {  // :289-332
  std::vector<Matrix> RVec;
  std::vector<Vector> tVec;
  collectNeighborTransforms(poseDict, RVec, tVec);
  if (RVec.empty()) throw std::runtime_error("no shared loop closure with this neighbor");
  Matrix ROpt;
  Vector tOpt;
  std::vector<size_t> inliers;
  // robust single rotation averaging with a ~30 deg chordal threshold, unit kappa
  robustSingleRotationAveraging(ROpt, inliers, RVec, Vector(), angular2ChordalSO3(0.5));
  if (mParams.verbose)
    std::printf("[RobustRelativeTransform] This robot %u, neighbor %u: finds %zu inliers out of %zu measurements.\n",
                mID, neighborID, inliers.size(), RVec.size());
  if (inliers.empty()) throw std::runtime_error("Robust single rotation averaging returns empty inlier set!");
  std::vector<Vector> tIn;
  for (size_t i : inliers) tIn.push_back(tVec[i]);
  singleTranslationAveraging(tOpt, tIn);
  Matrix T = Matrix::Identity(d + 1, d + 1);
  T.setBlock(0, 0, ROpt);
  T.setBlock(0, d, tOpt);
  return T;
}

Matrix PGOAgent::computeRobustNeighborTransform(unsigned neighborID, const PoseDict& poseDict) {  // :334-367
  std::vector<Matrix> RVec;
  std::vector<Vector> tVec;
  collectNeighborTransforms(poseDict, RVec, tVec);
  if (RVec.empty()) throw std::runtime_error("no shared loop closure with this neighbor");
  const size_t m = RVec.size();
  Vector kappa(static_cast<long>(m), 1), tau(static_cast<long>(m), 1);
  for (size_t i = 0; i < m; ++i) {
    kappa(static_cast<long>(i), 0) = 1.82;  // rotation stddev ~30 deg
    tau(static_cast<long>(i), 0) = 0.01;    // translation stddev 10 m
  }
  Matrix ROpt;
  Vector tOpt;
  std::vector<size_t> inliers;
  robustSinglePoseAveraging(ROpt, tOpt, inliers, RVec, tVec, kappa, tau,
                            RobustCost::computeErrorThresholdAtQuantile(0.9, 3));
  if (mParams.verbose)
    std::printf("[RobustRelativeTransform] This robot %u, neighbor %u: finds %zu inliers out of %zu measurements.\n",
                mID, neighborID, inliers.size(), m);
  if (inliers.empty()) throw std::runtime_error("Robust single pose averaging returns empty inlier set!");
  Matrix T = Matrix::Identity(d + 1, d + 1);
  T.setBlock(0, 0, ROpt);
  T.setBlock(0, d, tOpt);
  return T;
}

void PGOAgent::initializeInGlobalFrame(unsigned neighborID, const PoseDict& poseDict) {  // :369-432
  if (!YLift) throw std::logic_error("initializeInGlobalFrame: lifting matrix not set");
  neighborPoseDict.clear();
  neighborAuxPoseDict.clear();
  Matrix Tw2w1;
  try {
    Tw2w1 = computeRobustNeighborTransformTwoStage(neighborID, poseDict);
  } catch (const std::runtime_error&) {
    std::printf("Robust initialization is not successful! Abort and wait to try again...\n");
    return;
  }
  const long b = d + 1;
  Matrix T = *TLocalInit;
  Matrix Tw1f = Matrix::Identity(b, b);
  for (unsigned i = 0; i < n; ++i) {
    Tw1f.setBlock(0, 0, T.block(0, i * b, d, b));
    T.setBlock(0, i * b, (Tw2w1 * Tw1f).block(0, 0, d, b));
  }
  X = (*YLift) * T;
  XInit = X;
  mState = INITIALIZED;
  if (mParams.acceleration) initializeAcceleration();
}

void PGOAgent::updateNeighborPoses(unsigned neighborID, const PoseDict& poseDict) {  // :434-458
  const bool neighborInit = getNeighborStatus(neighborID).state == INITIALIZED;
  if (mState == WAIT_FOR_INITIALIZATION && neighborInit) initializeInGlobalFrame(neighborID, poseDict);
  for (const auto& kv : poseDict) {
    if (neighborSharedPoseIDs.find(kv.first) == neighborSharedPoseIDs.end()) continue;
    if (mState == INITIALIZED && neighborInit) neighborPoseDict[kv.first] = kv.second;
  }
}

void PGOAgent::updateAuxNeighborPoses(unsigned neighborID, const PoseDict& poseDict) {  // :460-479
  const bool neighborInit = getNeighborStatus(neighborID).state == INITIALIZED;
  for (const auto& kv : poseDict) {
    if (neighborSharedPoseIDs.find(kv.first) == neighborSharedPoseIDs.end()) continue;
    if (mState == INITIALIZED && neighborInit) neighborAuxPoseDict[kv.first] = kv.second;
  }
}

bool PGOAgent::getTrajectoryInLocalFrame(Matrix& Trajectory) {  // :481-498
  if (mState != INITIALIZED) return false;
  Matrix T = X.block(0, 0, r, d).transpose() * X;
  const Matrix t0 = T.block(0, d, d, 1);
  for (unsigned i = 0; i < n; ++i) {
    T.setBlock(0, i * (d + 1), projectToRotationGroup(T.block(0, i * (d + 1), d, d)));
    T.setBlock(0, i * (d + 1) + d, T.block(0, i * (d + 1) + d, d, 1) - t0);
  }
  Trajectory = T;
  return true;
}

void PGOAgent::constructQMatrix() {  // :720-781
  std::vector<RelativeSEMeasurement> priv = odometry;
  priv.insert(priv.end(), privateLoopClosures.begin(), privateLoopClosures.end());
  std::vector<std::pair<std::pair<int, int>, double>> extra;
  const SparseMatrix Qp = constructConnectionLaplacianSE(priv, n);
  const unsigned b = d + 1;
  std::vector<std::pair<std::pair<int, int>, double>> trip;
  for (long i = 0; i < Qp.rows(); ++i)
    for (int k = Qp.outerIndexPtr()[i]; k < Qp.outerIndexPtr()[i + 1]; ++k)
      trip.push_back({{static_cast<int>(i), Qp.innerIndexPtr()[k]}, Qp.valuePtr()[k]});
  for (const auto& m : sharedLoopClosures) {
    Matrix T = Matrix::Zero(b, b), Om = Matrix::Zero(b, b);
    T.setBlock(0, 0, m.R);
    T.setBlock(0, d, m.t);
    T(d, d) = 1;
    for (unsigned u = 0; u < d; ++u) Om(u, u) = m.weight * m.kappa;
    Om(d, d) = m.weight * m.tau;
    const bool outgoing = m.r1 == mID;
    const size_t idx = outgoing ? m.p1 : m.p2;
    const Matrix W = outgoing ? T * Om * T.transpose() : Om;
    for (unsigned c = 0; c < b; ++c)
      for (unsigned rr = 0; rr < b; ++rr)
        trip.push_back({{static_cast<int>(idx * b + rr), static_cast<int>(idx * b + c)}, W(rr, c)});
  }
  SparseMatrix Q(static_cast<long>(b * n), static_cast<long>(b * n));
  Q.setFromTriplets(trip);
  mProblem->setQ(Q);
}

bool PGOAgent::constructGMatrix(const PoseDict& poseDict) {  // :783-859
  const unsigned b = d + 1;
  std::vector<std::pair<std::pair<int, int>, double>> trip;
  for (const auto& m : sharedLoopClosures) {
    Matrix T = Matrix::Zero(b, b), Om = Matrix::Zero(b, b);
    T.setBlock(0, 0, m.R);
    T.setBlock(0, d, m.t);
    T(d, d) = 1;
    for (unsigned u = 0; u < d; ++u) Om(u, u) = m.weight * m.kappa;
    Om(d, d) = m.weight * m.tau;
    const bool outgoing = m.r1 == mID;
    const PoseID nID = outgoing ? PoseID(m.r2, m.p2) : PoseID(m.r1, m.p1);
    auto it = poseDict.find(nID);
    if (it == poseDict.end()) {
      if (mParams.verbose)
        std::printf("constructGMatrix: robot %u cannot find neighbor pose (%u, %u)\n", mID, nID.first, nID.second);
      return false;
    }
    const Matrix L = outgoing ? -(it->second * Om * T.transpose()) : -(it->second * T * Om);
    const size_t idx = outgoing ? m.p1 : m.p2;
    for (unsigned c = 0; c < b; ++c)
      for (unsigned rr = 0; rr < r; ++rr) trip.push_back({{static_cast<int>(rr), static_cast<int>(idx * b + c)}, L(rr, c)});
  }
  SparseMatrix G(r, static_cast<long>(b * n));
  G.setFromTriplets(trip);
  mProblem->setG(G);
  return true;
}

bool PGOAgent::updateX(bool doOptimization, bool acceleration) {  // :1093-1165
  if (!doOptimization) {
    if (acceleration) X = Y;
    return true;
  }
  if (mParams.robustCostType != RobustCostType::L2) constructQMatrix();
  const bool hasG = constructGMatrix(acceleration ? neighborAuxPoseDict : neighborPoseDict);
  if (!hasG) return false;
  QuadraticOptimizer optimizer(mProblem.get());
  optimizer.setVerbose(mParams.verbose);
  optimizer.setAlgorithm(mParams.algorithm);
  optimizer.setTrustRegionTolerance(1e-2);
  optimizer.setTrustRegionIterations(1);
  optimizer.setTrustRegionMaxInnerIterations(10);
  optimizer.setTrustRegionInitialRadius(100);
  X = optimizer.optimize(acceleration ? Y : X);
  mLastResult = optimizer.getOptResult();
  return true;
}

void PGOAgent::initializeAcceleration() {  // :1062-1071
  if (mState == INITIALIZED) {
    XPrev = X;
    gamma = 0;
    alpha = 0;
    V = X;
    Y = X;
  }
}

void PGOAgent::updateGamma() {
  const double N = mParams.numRobots;
  gamma = (1 + std::sqrt(1 + 4 * N * N * gamma * gamma)) / (2 * N);
}
void PGOAgent::updateAlpha() { alpha = 1 / (gamma * mParams.numRobots); }

void PGOAgent::updateY() {
  LiftedSEManifold M(r, d, n);
  Y = M.project((1 - alpha) * X + alpha * V);
}

void PGOAgent::updateV() {
  LiftedSEManifold M(r, d, n);
  V = M.project(V + gamma * (X - Y));
}

bool PGOAgent::shouldRestart() const {
  return mParams.acceleration && ((mIterationNumber + 1) % mParams.restartInterval == 0);
}

void PGOAgent::restartNesterovAcceleration(bool doOptimization) {  // :1040-1060
  if (mParams.acceleration && mState == INITIALIZED) {
    X = XPrev;
    updateX(doOptimization, false);
    V = X;
    Y = X;
    gamma = 0;
    alpha = 0;
  }
}

bool PGOAgent::shouldUpdateLoopClosureWeights() const {  // :1174-1179
  if (mParams.robustCostType == RobustCostType::L2) return false;
  return (mIterationNumber + 1) % mParams.robustOptInnerIters == 0;
}

void PGOAgent::updateLoopClosuresWeights() {  // :1181-1240
  const unsigned b = d + 1;
  for (auto& m : privateLoopClosures) {
    if (m.isKnownInlier) continue;
    const double res = std::sqrt(computeMeasurementError(m, X.block(0, m.p1 * b, r, d), X.block(0, m.p1 * b + d, r, 1),
                                                         X.block(0, m.p2 * b, r, d), X.block(0, m.p2 * b + d, r, 1)));
    m.weight = mRobustCost.weight(res);
  }
  for (auto& m : sharedLoopClosures) {
    if (m.isKnownInlier) continue;
    Matrix Y1, p1, Y2, p2;
    if (m.r1 == mID) {
      if (m.r2 < mID) continue;
      auto it = neighborPoseDict.find({static_cast<unsigned>(m.r2), static_cast<unsigned>(m.p2)});
      if (it == neighborPoseDict.end()) continue;
      Y1 = X.block(0, m.p1 * b, r, d);
      p1 = X.block(0, m.p1 * b + d, r, 1);
      Y2 = it->second.block(0, 0, r, d);
      p2 = it->second.block(0, d, r, 1);
    } else {
      if (m.r1 < mID) continue;
      auto it = neighborPoseDict.find({static_cast<unsigned>(m.r1), static_cast<unsigned>(m.p1)});
      if (it == neighborPoseDict.end()) continue;
      Y2 = X.block(0, m.p2 * b, r, d);
      p2 = X.block(0, m.p2 * b + d, r, 1);
      Y1 = it->second.block(0, 0, r, d);
      p1 = it->second.block(0, d, r, 1);
    }
    m.weight = mRobustCost.weight(std::sqrt(computeMeasurementError(m, Y1, p1, Y2, p2)));
  }
}

double PGOAgent::computeConvergedLoopClosureRatio() const {  // :1242-1280
  if (mParams.robustCostType != RobustCostType::GNC_TLS) return 1.0;
  double total = 0, converged = 0;
  for (const auto* lst : {&privateLoopClosures, &sharedLoopClosures})
    for (const auto& m : *lst) {
      if (m.isKnownInlier) continue;
      if (m.weight == 1 || m.weight == 0) converged += 1;
      total += 1;
    }
  return total > 0 ? converged / total : 1.0;
}

void PGOAgent::iterate(bool doOptimization) {  // :642-718
  mIterationNumber++;
  if (shouldUpdateLoopClosureWeights()) {
    updateLoopClosuresWeights();
    mRobustCost.update();
    if (!mParams.robustOptWarmStart && XInit) X = *XInit;
    if (mParams.acceleration) initializeAcceleration();
  }
  if (mState != INITIALIZED) return;
  XPrev = X;
  bool success;
  if (mParams.acceleration) {
    updateGamma();
    updateAlpha();
    updateY();
    success = updateX(doOptimization, true);
    updateV();
    if (shouldRestart()) restartNesterovAcceleration(doOptimization);
  } else {
    success = updateX(doOptimization, false);
  }
  if (doOptimization) {
    mStatus.agentID = mID;
    mStatus.state = mState;
    mStatus.iterationNumber = mIterationNumber;
    mStatus.relativeChange = std::sqrt((X - XPrev).squaredNorm() / n);
    bool ready = success && mStatus.relativeChange <= mParams.relChangeTol;
    if (computeConvergedLoopClosureRatio() < mParams.robustOptMinConvergenceRatio) ready = false;
    mStatus.readyToTerminate = ready;
  }
}

Matrix PGOAgent::localPoseGraphOptimization() {  // :964-990
  if (!TLocalInit) TLocalInit = odometryInitialization(d, n, odometry);
  std::vector<RelativeSEMeasurement> meas = odometry;
  meas.insert(meas.end(), privateLoopClosures.begin(), privateLoopClosures.end());
  QuadraticProblem problem(n, d, d);
  problem.setQ(constructConnectionLaplacianSE(meas, n));
  QuadraticOptimizer optimizer(&problem);
  optimizer.setVerbose(mParams.verbose);
  optimizer.setTrustRegionInitialRadius(10);
  optimizer.setTrustRegionIterations(10);
  optimizer.setTrustRegionTolerance(1e-1);
  optimizer.setTrustRegionMaxInnerIterations(50);
  Matrix Topt = optimizer.optimize(*TLocalInit);
  mLastResult = optimizer.getOptResult();
  return Topt;
}

}  // namespace DPGO
