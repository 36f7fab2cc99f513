@echo off
REM Smoke-test a running deployment (Windows twin of scripts/test-deployment.sh).
setlocal
set URL=%1
if "%URL%"=="" set URL=http://localhost:8000
echo health:
curl -fs %URL%/health || exit /b 1
echo.
echo regions:
curl -fs %URL%/regions || exit /b 1
echo.
echo queue:
curl -fs %URL%/api/v1/jobs/stats/queue || exit /b 1
echo.
echo workers:
curl -fs %URL%/api/v1/workers || exit /b 1
echo.
set BODY={\"type\":\"llm\",\"params\":{\"messages\":[{\"role\":\"user\",\"content\":\"hello\"}],\"max_tokens\":16,\"temperature\":0}}
for /f %%c in ('curl -s -o "%TEMP%\dgi_job.json" -w "%%{http_code}" -X POST "%URL%/api/v1/jobs/sync?timeout=120&wait_for_worker=false" -H "Content-Type: application/json" -d "%BODY%"') do set CODE=%%c
echo sync job HTTP %CODE%
type "%TEMP%\dgi_job.json"
echo.
if "%CODE%"=="200" exit /b 0
if "%CODE%"=="503" exit /b 0
exit /b 1
