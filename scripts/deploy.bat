@echo off
REM Deploy the control plane with docker compose (Windows twin of scripts/deploy.sh).
REM   scripts\deploy.bat server   - postgres + redis + API server
REM   scripts\deploy.bat worker   - not supported on Windows hosts (the worker needs ROCm /dev/kfd)
setlocal
cd /d "%~dp0\.."
set MODE=%1
if "%MODE%"=="" set MODE=server
where docker >nul 2>nul || (echo docker is required & exit /b 1)
if not exist .env (echo no .env: using defaults from .env.example & copy .env.example .env >nul)
if /I "%MODE%"=="server" (
  docker compose up -d --build postgres redis server || exit /b 1
) else if /I "%MODE%"=="worker" (
  echo The MI355X worker needs a Linux host with ROCm ^(/dev/kfd, /dev/dri^); run scripts/deploy.sh worker there.
  exit /b 1
) else (
  echo usage: %~nx0 [server^|worker]
  exit /b 2
)
set PORT=8000
for /f "tokens=2 delims==" %%p in ('findstr /b "SERVER_PORT=" .env') do set PORT=%%p
for /l %%i in (1,1,30) do (
  curl -fs http://localhost:%PORT%/health >nul 2>nul && (echo server healthy on :%PORT% & exit /b 0)
  timeout /t 2 /nobreak >nul
)
echo server did not become healthy
docker compose logs --tail=50 server
exit /b 1
